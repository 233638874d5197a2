"""Live Cassandra interop over the CQL native protocol (v4), no driver needed.

The reference writes its rows through the DataStax driver (CassandraOpService.scala:
insertMessage / insertQueueMsg / ... over a session).  This broker keeps those rows in its
embedded WAL store; this module talks to a live Cassandra node directly:

* ``CqlClient``          — one connection: STARTUP (+ PasswordAuthenticator), QUERY with bound
                           values, PREPARE / EXECUTE, BATCH, result rows decoded by column type
* ``push(store, client)`` — the store's live rows into the keyspace (DDL first, then every
                           table's rows as batched prepared INSERTs) -- a running broker's
                           state mirrored into a Cassandra cluster
* ``pull(client, store)`` — the keyspace's rows into a store (the reverse: start a broker from
                           a Cassandra-resident state)

Frames: ``version | flags | stream (i16) | opcode | length (i32)`` then the body, big
endian throughout (native_protocol_v4.spec sections 2-4).  One request in flight per
connection (stream 0); no compression, no tracing.
"""

import socket
import struct

from .cql import ORDER, SCHEMA, _insert, ddl, rows

# opcodes
ERROR, STARTUP, READY, AUTHENTICATE, OPTIONS, SUPPORTED, QUERY, RESULT = 0, 1, 2, 3, 5, 6, 7, 8
PREPARE, EXECUTE, REGISTER, EVENT, BATCH, AUTH_CHALLENGE, AUTH_RESPONSE, AUTH_SUCCESS = 9, 10, 11, 12, 13, 14, 15, 16
# result kinds
R_VOID, R_ROWS, R_KEYSPACE, R_PREPARED, R_SCHEMA = 1, 2, 3, 4, 5
# consistency levels
ONE, QUORUM, LOCAL_QUORUM = 0x0001, 0x0004, 0x0006
# column type option ids
T_CUSTOM, T_ASCII, T_BIGINT, T_BLOB, T_BOOLEAN, T_INT, T_VARCHAR, T_LIST, T_MAP, T_SET = (
    0x0000, 0x0001, 0x0002, 0x0003, 0x0004, 0x0009, 0x000D, 0x0020, 0x0021, 0x0022)
_TYPE_IDS = {"bigint": T_BIGINT, "int": T_INT, "boolean": T_BOOLEAN, "blob": T_BLOB, "text": T_VARCHAR,
             "varchar": T_VARCHAR, "ascii": T_ASCII}


class CqlError(Exception):
    def __init__(self, code, msg):
        super().__init__(f"CQL error 0x{code:04x}: {msg}")
        self.code = code


# ---------------------------------------------------------------------------- primitives
def _short(n):
    return struct.pack(">H", n)


def _int(n):
    return struct.pack(">i", n)


def _string(s):
    b = s.encode()
    return _short(len(b)) + b


def _long_string(s):
    b = s.encode()
    return _int(len(b)) + b


def _bytes(b):
    return _int(-1) if b is None else _int(len(b)) + b


def _string_map(m):
    return _short(len(m)) + b"".join(_string(k) + _string(v) for k, v in m.items())


class _Reader:
    def __init__(self, b):
        self.b, self.p = b, 0

    def take(self, n):
        v = self.b[self.p:self.p + n]
        if len(v) != n:
            raise CqlError(0, "truncated frame body")
        self.p += n
        return v

    def byte(self):
        return self.take(1)[0]

    def short(self):
        return struct.unpack(">H", self.take(2))[0]

    def int(self):
        return struct.unpack(">i", self.take(4))[0]

    def string(self):
        return self.take(self.short()).decode()

    def bytes(self):
        n = self.int()
        return None if n < 0 else self.take(n)

    def short_bytes(self):
        return self.take(self.short())

    def option(self):
        t = self.short()
        if t == T_CUSTOM:
            return (t, self.string())
        if t in (T_LIST, T_SET):
            return (t, self.option())
        if t == T_MAP:
            return (t, self.option(), self.option())
        return (t,)


# ---------------------------------------------------------------------------- values
def encode_value(v, ty):
    """A Python value as the [bytes] of CQL type ``ty`` (schema spelling: bigint, int,
    boolean, blob, text, set<text>, map<text, text>)."""
    if v is None:
        return None
    ty = ty.replace(" ", "")
    if ty == "bigint":
        return struct.pack(">q", int(v))
    if ty == "int":
        return struct.pack(">i", int(v))
    if ty == "boolean":
        return b"\x01" if v else b"\x00"
    if ty == "blob":
        return bytes(v)
    if ty in ("text", "varchar", "ascii"):
        return str(v).encode()
    if ty.startswith("set<") or ty.startswith("list<"):
        inner = ty[ty.index("<") + 1:-1]
        items = sorted(v) if ty.startswith("set<") else list(v)
        return _int(len(items)) + b"".join(_bytes(encode_value(x, inner)) for x in items)
    if ty.startswith("map<"):
        kt, vt = ty[4:-1].split(",", 1)
        return _int(len(v)) + b"".join(_bytes(encode_value(k, kt)) + _bytes(encode_value(x, vt))
                                       for k, x in sorted(v.items()))
    raise ValueError(f"unsupported CQL type {ty}")


def decode_value(b, opt):
    if b is None:
        return None
    t = opt[0]
    if t == T_BIGINT:
        return struct.unpack(">q", b)[0]
    if t == T_INT:
        return struct.unpack(">i", b)[0]
    if t == T_BOOLEAN:
        return b != b"\x00"
    if t == T_BLOB:
        return bytes(b)
    if t in (T_VARCHAR, T_ASCII):
        return b.decode()
    if t in (T_SET, T_LIST):
        r = _Reader(b)
        items = [decode_value(r.bytes(), opt[1]) for _ in range(r.int())]
        return set(items) if t == T_SET else items
    if t == T_MAP:
        r = _Reader(b)
        out = {}
        for _ in range(r.int()):
            k = decode_value(r.bytes(), opt[1])
            out[k] = decode_value(r.bytes(), opt[2])
        return out
    return bytes(b)   # (other types: raw bytes)


# ---------------------------------------------------------------------------- client
class CqlClient:
    """One CQL native-protocol v4 connection (blocking, stream 0)."""

    def __init__(self, host="127.0.0.1", port=9042, user=None, password=None, timeout=10.0):
        self.sock = socket.create_connection((host, port), timeout=timeout)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self._prepared = {}
        op, body = self._request(STARTUP, _string_map({"CQL_VERSION": "3.0.0"}))
        if op == AUTHENTICATE:
            if user is None:
                raise CqlError(0x0100, "server requires authentication")
            token = b"\x00" + user.encode() + b"\x00" + (password or "").encode()   # SASL PLAIN
            op, body = self._request(AUTH_RESPONSE, _bytes(token))
            if op != AUTH_SUCCESS:
                raise CqlError(0x0100, f"authentication failed (opcode {op})")
        elif op != READY:
            raise CqlError(0, f"unexpected STARTUP answer opcode {op}")

    def close(self):
        try:
            self.sock.close()
        except OSError:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- framing
    def _recv(self, n):
        buf = b""
        while len(buf) < n:
            k = self.sock.recv(n - len(buf))
            if not k:
                raise CqlError(0, "connection closed by the server")
            buf += k
        return buf

    def _request(self, opcode, body):
        self.sock.sendall(struct.pack(">BBhBi", 0x04, 0, 0, opcode, len(body)) + body)
        ver, _flags, _stream, op, n = struct.unpack(">BBhBi", self._recv(9))
        if ver != 0x84:
            raise CqlError(0, f"unexpected protocol version 0x{ver:02x}")
        body = self._recv(n)
        if op == ERROR:
            r = _Reader(body)
            code = r.int()
            raise CqlError(code, r.string())
        return op, body

    @staticmethod
    def _params(consistency, values):
        if not values:
            return _short(consistency) + b"\x00"
        return _short(consistency) + b"\x01" + _short(len(values)) + b"".join(_bytes(v) for v in values)

    # -- results
    @staticmethod
    def _result(body):
        r = _Reader(body)
        kind = r.int()
        if kind == R_ROWS:
            flags = r.int()
            ncol = r.int()
            if flags & 0x0002:   # has more pages: paging state
                r.bytes()
            cols = []
            if not flags & 0x0004:   # metadata present
                glob = flags & 0x0001
                if glob:
                    r.string(), r.string()
                for _ in range(ncol):
                    if not glob:
                        r.string(), r.string()
                    cols.append((r.string(), r.option()))
            out = []
            for _ in range(r.int()):
                out.append({name: decode_value(r.bytes(), opt) for name, opt in cols})
            return out
        if kind == R_PREPARED:
            return r.short_bytes()
        if kind == R_KEYSPACE:
            return r.string()
        return None

    # -- requests
    def query(self, cql, values=(), consistency=ONE):
        """Run one statement; ``values`` are already-encoded [bytes] for its ``?``
        markers.  Returns rows (list of dicts) for a SELECT, else None."""
        _, body = self._request(QUERY, _long_string(cql) + self._params(consistency, list(values)))
        return self._result(body)

    def prepare(self, cql):
        qid = self._prepared.get(cql)
        if qid is None:
            _, body = self._request(PREPARE, _long_string(cql))
            qid = self._prepared[cql] = self._result(body)
        return qid

    def execute(self, cql, values=(), consistency=ONE):
        _, body = self._request(EXECUTE, _short(len(self.prepare(cql))) + self.prepare(cql)
                                + self._params(consistency, list(values)))
        return self._result(body)

    def batch(self, stmts, consistency=ONE, logged=False):
        """(cql, values) pairs as one BATCH of prepared statements."""
        parts = []
        for cql, values in stmts:
            qid = self.prepare(cql)
            parts.append(b"\x01" + _short(len(qid)) + qid + _short(len(values)) + b"".join(_bytes(v) for v in values))
        body = bytes([0 if logged else 1]) + _short(len(parts)) + b"".join(parts) + _short(consistency) + b"\x00"
        self._request(BATCH, body)


# ---------------------------------------------------------------------------- store <-> cluster
def _insert_cql(keyspace, table):
    cols = [c for c, _ in SCHEMA[table][0]]
    return f"INSERT INTO {keyspace}.{table} ({', '.join(cols)}) VALUES ({', '.join('?' * len(cols))})"


def push(store, client, keyspace="chanamq", replication=1, batch=64, consistency=ONE):
    """The store's live rows into ``keyspace`` (created first); returns rows per table."""
    for stmt in ddl(keyspace, replication).split(";"):
        stmt = stmt.strip()
        if stmt and not stmt.upper().startswith("USE "):
            if stmt.upper().startswith("CREATE TABLE"):
                stmt = stmt.replace("CREATE TABLE IF NOT EXISTS ", f"CREATE TABLE IF NOT EXISTS {keyspace}.", 1)
            client.query(stmt, consistency=consistency)
    data = rows(store)
    n = {}
    for t in ORDER:
        cols = SCHEMA[t][0]
        cql = _insert_cql(keyspace, t)
        pend = []
        for r in data[t]:
            pend.append((cql, [encode_value(r.get(c), ty) for c, ty in cols]))
            if len(pend) == batch:
                client.batch(pend, consistency)
                pend = []
        if pend:
            client.batch(pend, consistency)
        n[t] = len(data[t])
    return n


def pull(client, store, keyspace="chanamq", consistency=ONE):
    """Every row of ``keyspace``'s tables into ``store``; returns rows per table."""
    n = {}
    for t in ORDER:
        got = client.query(f"SELECT * FROM {keyspace}.{t}", consistency=consistency) or []
        for r in got:
            for c, ty in SCHEMA[t][0]:   # absent collections read back as empty
                if r.get(c) is None and (ty.startswith("set") or ty.startswith("map")):
                    r[c] = set() if ty.startswith("set") else {}
            _insert(store, t, r)
        n[t] = len(got)
    store.sync()
    return n


__all__ = ["CqlClient", "CqlError", "push", "pull", "encode_value", "decode_value"]
