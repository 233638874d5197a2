"""A minimal CQL native-protocol v4 server for tests (no Cassandra in this environment):
STARTUP (optionally PasswordAuthenticator), QUERY / PREPARE / EXECUTE / BATCH for the
statements chanamq_amd/store/cql_native.py sends -- CREATE KEYSPACE / TABLE (accepted),
``INSERT INTO ks.t (cols) VALUES (?, ...)`` (rows kept per table, last write wins per
primary key) and ``SELECT * FROM ks.t`` (rows returned with column metadata).  Column
types come from the reference schema (chanamq_amd/store/cql.py SCHEMA), so the server
decodes and re-encodes values independently of the client's codec tables."""

import re
import socket
import struct
import threading

from chanamq_amd.store.cql import SCHEMA

_OPT = {"bigint": b"\x00\x02", "int": b"\x00\x09", "boolean": b"\x00\x04", "blob": b"\x00\x03",
        "text": b"\x00\x0d"}


def _opt(ty):
    ty = ty.replace(" ", "")
    if ty.startswith("set<"):
        return b"\x00\x22" + _opt(ty[4:-1])
    if ty.startswith("map<"):
        k, v = ty[4:-1].split(",", 1)
        return b"\x00\x21" + _opt(k) + _opt(v)
    return _OPT[ty]


def _dec(b, ty):   # the server's own decoder (not the client's)
    ty = ty.replace(" ", "")
    if b is None:
        return None
    if ty == "bigint":
        return struct.unpack(">q", b)[0]
    if ty == "int":
        return struct.unpack(">i", b)[0]
    if ty == "boolean":
        return b[0] != 0
    if ty == "blob":
        return bytes(b)
    if ty == "text":
        return b.decode()
    p, n = 4, struct.unpack(">i", b[:4])[0]
    items = []
    for _ in range(n * (2 if ty.startswith("map<") else 1)):
        ln = struct.unpack(">i", b[p:p + 4])[0]
        items.append(b[p + 4:p + 4 + ln])
        p += 4 + ln
    if ty.startswith("set<"):
        return frozenset(_dec(x, ty[4:-1]) for x in items)
    kt, vt = ty[4:-1].split(",", 1)
    return tuple(sorted((_dec(items[i], kt), _dec(items[i + 1], vt)) for i in range(0, len(items), 2)))


def _enc(v, ty):
    ty = ty.replace(" ", "")
    if v is None:
        return struct.pack(">i", -1)
    if ty == "bigint":
        b = struct.pack(">q", v)
    elif ty == "int":
        b = struct.pack(">i", v)
    elif ty == "boolean":
        b = b"\x01" if v else b"\x00"
    elif ty == "blob":
        b = bytes(v)
    elif ty == "text":
        b = v.encode()
    elif ty.startswith("set<"):
        b = struct.pack(">i", len(v)) + b"".join(_enc(x, ty[4:-1]) for x in sorted(v))
    else:
        kt, vt = ty[4:-1].split(",", 1)
        b = struct.pack(">i", len(v)) + b"".join(_enc(k, kt) + _enc(x, vt) for k, x in v)
    return struct.pack(">i", len(b)) + b


class FakeCql:
    def __init__(self, user=None, password=None):
        self.user, self.password = user, password
        self.tables = {}          # (ks, table) -> {pk tuple: row dict}
        self.statements = []      # every statement text seen
        self.prepared = {}
        self.lock = threading.Lock()
        self.ls = socket.socket()
        self.ls.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.ls.bind(("127.0.0.1", 0))
        self.ls.listen(8)
        self.port = self.ls.getsockname()[1]
        self._stop = False
        threading.Thread(target=self._accept, daemon=True).start()

    def close(self):
        self._stop = True
        self.ls.close()

    def _accept(self):
        while not self._stop:
            try:
                c, _ = self.ls.accept()
            except OSError:
                return
            threading.Thread(target=self._serve, args=(c,), daemon=True).start()

    @staticmethod
    def _recv(c, n):
        buf = b""
        while len(buf) < n:
            k = c.recv(n - len(buf))
            if not k:
                raise EOFError
            buf += k
        return buf

    def _send(self, c, stream, op, body):
        c.sendall(struct.pack(">BBhBi", 0x84, 0, stream, op, len(body)) + body)

    def _error(self, c, stream, code, msg):
        m = msg.encode()
        self._send(c, stream, 0, struct.pack(">iH", code, len(m)) + m)

    def _serve(self, c):
        try:
            while True:
                ver, _f, stream, op, n = struct.unpack(">BBhBi", self._recv(c, 9))
                body = self._recv(c, n)
                assert ver == 0x04, ver
                try:
                    self._handle(c, stream, op, body)
                except Exception as e:   # noqa: BLE001 - reported to the client
                    self._error(c, stream, 0x2200, repr(e))
        except (EOFError, OSError):
            c.close()

    def _values(self, body, p):
        cons, flags = struct.unpack(">HB", body[p:p + 3])
        p += 3
        vals = []
        if flags & 1:
            k = struct.unpack(">H", body[p:p + 2])[0]
            p += 2
            for _ in range(k):
                ln = struct.unpack(">i", body[p:p + 4])[0]
                vals.append(None if ln < 0 else body[p + 4:p + 4 + ln])
                p += 4 + max(ln, 0)
        return vals, p

    def _run(self, cql, vals):
        with self.lock:
            self.statements.append(cql)
        s = cql.strip()
        m = re.match(r"INSERT INTO (\w+)\.(\w+) \(([^)]*)\) VALUES", s)
        if m:
            ks, t, cols = m.group(1), m.group(2), [x.strip() for x in m.group(3).split(",")]
            types = dict(SCHEMA[t][0])
            row = {col: _dec(v, types[col]) for col, v in zip(cols, vals)}
            pk = tuple(row[k] for k in SCHEMA[t][1] + SCHEMA[t][2])
            with self.lock:
                self.tables.setdefault((ks, t), {})[pk] = row
            return struct.pack(">i", 1)
        m = re.match(r"DELETE FROM (\w+)\.(\w+) WHERE (.+)$", s)
        if m:   # a row (every key column given) or a whole partition (a key prefix)
            ks, t = m.group(1), m.group(2)
            conds = [x.strip() for x in m.group(3).split(" AND ")]
            cols = [c.split("=")[0].strip() for c in conds]
            types = dict(SCHEMA[t][0])
            want = {col: _dec(v, types[col]) for col, v in zip(cols, vals)}
            keys = SCHEMA[t][1] + SCHEMA[t][2]
            assert cols == keys[:len(cols)] and len(cols) >= len(SCHEMA[t][1]), ("not a key prefix", cols)
            with self.lock:
                tab = self.tables.setdefault((ks, t), {})
                for pk in [pk for pk in tab if pk[:len(cols)] == tuple(want[c] for c in cols)]:
                    del tab[pk]
            return struct.pack(">i", 1)
        m = re.match(r"SELECT \* FROM (\w+)\.(\w+)$", s)
        if m:
            ks, t = m.group(1), m.group(2)
            cols = SCHEMA[t][0]
            with self.lock:
                data = list(self.tables.get((ks, t), {}).values())
            out = struct.pack(">iii", 2, 1, len(cols))
            for x in (ks, t):
                out += struct.pack(">H", len(x)) + x.encode()
            for col, ty in cols:
                out += struct.pack(">H", len(col)) + col.encode() + _opt(ty)
            out += struct.pack(">i", len(data))
            for r in data:
                out += b"".join(_enc(r.get(col), ty) for col, ty in cols)
            return out
        if s.upper().startswith("CREATE "):
            return struct.pack(">i", 1)
        raise ValueError("unsupported statement: " + s[:60])

    def _handle(self, c, stream, op, body):
        if op == 1:   # STARTUP
            if self.user is not None:
                a = b"org.apache.cassandra.auth.PasswordAuthenticator"
                self._send(c, stream, 3, struct.pack(">H", len(a)) + a)
            else:
                self._send(c, stream, 2, b"")
        elif op == 15:   # AUTH_RESPONSE: SASL PLAIN
            ln = struct.unpack(">i", body[:4])[0]
            _, u, pw = body[4:4 + ln].split(b"\x00")
            if u.decode() == self.user and pw.decode() == self.password:
                self._send(c, stream, 16, struct.pack(">i", -1))
            else:
                self._error(c, stream, 0x0100, "bad credentials")
        elif op == 7:   # QUERY
            ln = struct.unpack(">i", body[:4])[0]
            cql = body[4:4 + ln].decode()
            vals, _ = self._values(body, 4 + ln)
            self._send(c, stream, 8, self._run(cql, vals))
        elif op == 9:   # PREPARE
            ln = struct.unpack(">i", body[:4])[0]
            cql = body[4:4 + ln].decode()
            qid = struct.pack(">I", len(self.prepared) + 1)
            with self.lock:
                self.prepared[qid] = cql
            # kind, id, (empty) variables metadata, (empty) result metadata
            self._send(c, stream, 8, struct.pack(">iH", 4, len(qid)) + qid + struct.pack(">iii", 0, 0, 0)
                       + struct.pack(">ii", 4, 0))
        elif op == 10:   # EXECUTE
            ln = struct.unpack(">H", body[:2])[0]
            cql = self.prepared[body[2:2 + ln]]
            vals, _ = self._values(body, 2 + ln)
            self._send(c, stream, 8, self._run(cql, vals))
        elif op == 13:   # BATCH
            p = 1
            n = struct.unpack(">H", body[p:p + 2])[0]
            p += 2
            for _ in range(n):
                kind = body[p]
                p += 1
                assert kind == 1
                ln = struct.unpack(">H", body[p:p + 2])[0]
                cql = self.prepared[body[p + 2:p + 2 + ln]]
                p += 2 + ln
                k = struct.unpack(">H", body[p:p + 2])[0]
                p += 2
                vals = []
                for _ in range(k):
                    vl = struct.unpack(">i", body[p:p + 4])[0]
                    vals.append(None if vl < 0 else body[p + 4:p + 4 + vl])
                    p += 4 + max(vl, 0)
                self._run(cql, vals)
            self._send(c, stream, 8, struct.pack(">i", 1))
        else:
            self._error(c, stream, 0x000A, f"opcode {op} not supported by the fake server")
