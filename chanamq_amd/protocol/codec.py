"""Golden (reference-semantics) AMQP 0-9-1 codec in pure Python.

This is the bit-exact model the C++ host codec (csrc/core/codec.*) and the HIP
data-plane kernels (csrc/kernels/dataplane.hip) are tested against.  It is also
what the test client / load generator uses.

Reference behaviour pinned here (all paths under /root/reference):
  * bits pack LSB-first, flushed by any non-bit field
      chana-mq-base/.../method/ArgumentsWriter.scala:41-46,85-96; ArgumentsReader.scala:33-36,69-78
  * shortstr <= 255 bytes (ValueWriter.scala:46-54), longstr u32
  * timestamp travels as u64 seconds (ValueReader.scala:59, ValueWriter.scala:195-197)
  * field tables: tags S I D T F A b d f l s t x V, first duplicate key wins
      (ValueReader.scala:62-113, ValueWriter.scala:85-159)
  * content header: class u16 | weight u16 | body-size u64 | flags u16-chain | props
      (AMQContentHeader.scala:12-56, ContentHeaderPropertyWriter.scala:31-53)
  * body frames split at frame_max - 8 (AMQCommand.scala:49-59)
"""

import struct
from decimal import Decimal

from . import constants as C
from .methods import BASIC_PROPERTIES, BY_ID, BY_NAME


class CodecError(Exception):
    """Malformed input (maps to FRAME_ERROR / SYNTAX_ERROR on the wire)."""

    def __init__(self, msg, code=C.FRAME_ERROR):
        super().__init__(msg)
        self.code = code


class Typed:
    """Field value with an explicit wire tag (e.g. Typed('s', 5) for a short)."""

    __slots__ = ("tag", "value")

    def __init__(self, tag, value):
        self.tag, self.value = tag, value

    def __eq__(self, o):
        return isinstance(o, Typed) and (o.tag, o.value) == (self.tag, self.value)

    def __repr__(self):
        return f"Typed({self.tag!r}, {self.value!r})"


# --------------------------------------------------------------------------- writer
class Writer:
    __slots__ = ("buf", "_bits", "_nbits")

    def __init__(self):
        self.buf = bytearray()
        self._bits = 0
        self._nbits = 0

    def _flush(self):
        if self._nbits:
            self.buf.append(self._bits)
            self._bits = 0
            self._nbits = 0

    def bit(self, v):
        if self._nbits == 8:
            self._flush()
        if v:
            self._bits |= 1 << self._nbits
        self._nbits += 1

    def octet(self, v):
        self._flush()
        self.buf.append(v & 0xFF)

    def short(self, v):
        self._flush()
        self.buf += struct.pack(">H", v & 0xFFFF)

    def long(self, v):
        self._flush()
        self.buf += struct.pack(">I", v & 0xFFFFFFFF)

    def longlong(self, v):
        self._flush()
        self.buf += struct.pack(">Q", v & 0xFFFFFFFFFFFFFFFF)

    def timestamp(self, v):
        self.longlong(int(v))

    def shortstr(self, s):
        self._flush()
        b = s.encode("utf-8") if isinstance(s, str) else bytes(s)
        if len(b) > 255:
            raise CodecError("shortstr longer than 255 bytes", C.SYNTAX_ERROR)
        self.buf.append(len(b))
        self.buf += b

    def longstr(self, s):
        self._flush()
        b = s.encode("utf-8") if isinstance(s, str) else bytes(s)
        self.buf += struct.pack(">I", len(b))
        self.buf += b

    def table(self, t):
        self._flush()
        self.buf += encode_table(t or {})

    def getvalue(self):
        self._flush()
        return bytes(self.buf)


def _encode_value(w: bytearray, v):
    if isinstance(v, Typed):
        tag, v = v.tag, v.value
    elif v is None:
        tag = "V"
    elif isinstance(v, bool):
        tag = "t"
    elif isinstance(v, int):
        tag = "I" if -(2 ** 31) <= v < 2 ** 31 else "l"
    elif isinstance(v, float):
        tag = "d"
    elif isinstance(v, Decimal):
        tag = "D"
    elif isinstance(v, (str, bytes, bytearray)):
        tag = "S"
    elif isinstance(v, dict):
        tag = "F"
    elif isinstance(v, (list, tuple)):
        tag = "A"
    else:
        raise CodecError(f"cannot encode field value {type(v)}", C.SYNTAX_ERROR)
    w.append(ord(tag))
    if tag == "S":
        b = v.encode("utf-8") if isinstance(v, str) else bytes(v)
        w += struct.pack(">I", len(b)) + b
    elif tag == "x":
        b = bytes(v)
        w += struct.pack(">I", len(b)) + b
    elif tag == "I":
        w += struct.pack(">i", v)
    elif tag == "l":
        w += struct.pack(">q", v)
    elif tag == "s":
        w += struct.pack(">h", v)
    elif tag == "b":
        w += struct.pack(">b", v)
    elif tag == "B":
        w += struct.pack(">B", v)
    elif tag == "u":
        w += struct.pack(">H", v)
    elif tag == "i":
        w += struct.pack(">I", v)
    elif tag == "t":
        w.append(1 if v else 0)
    elif tag == "d":
        w += struct.pack(">d", v)
    elif tag == "f":
        w += struct.pack(">f", v)
    elif tag == "T":
        w += struct.pack(">Q", int(v))
    elif tag == "D":
        sign, digits, exp = Decimal(v).as_tuple()
        scale = max(0, -exp)
        unscaled = int(Decimal(v).scaleb(scale))
        w += struct.pack(">Bi", scale, unscaled)
    elif tag == "F":
        w += encode_table(v)
    elif tag == "A":
        inner = bytearray()
        for item in v:
            _encode_value(inner, item)
        w += struct.pack(">I", len(inner)) + inner
    elif tag == "V":
        pass
    else:
        raise CodecError(f"unknown field tag {tag!r}", C.SYNTAX_ERROR)


def encode_table(t) -> bytes:
    inner = bytearray()
    for k, v in t.items():
        kb = k.encode("utf-8") if isinstance(k, str) else bytes(k)
        if len(kb) > 255:
            raise CodecError("table key longer than 255 bytes", C.SYNTAX_ERROR)
        inner.append(len(kb))
        inner += kb
        _encode_value(inner, v)
    return struct.pack(">I", len(inner)) + bytes(inner)


# --------------------------------------------------------------------------- reader
class Reader:
    __slots__ = ("data", "pos", "end", "_bits", "_nbits")

    def __init__(self, data, pos=0, end=None):
        self.data = data
        self.pos = pos
        self.end = len(data) if end is None else end
        self._bits = 0
        self._nbits = 0

    def _need(self, n):
        if self.pos + n > self.end:
            raise CodecError("truncated input", C.FRAME_ERROR)

    def _clear(self):
        self._nbits = 0

    def bit(self):
        if self._nbits == 0:
            self._need(1)
            self._bits = self.data[self.pos]
            self.pos += 1
            self._nbits = 8
        v = bool(self._bits & 1)
        self._bits >>= 1
        self._nbits -= 1
        return v

    def octet(self):
        self._clear()
        self._need(1)
        v = self.data[self.pos]
        self.pos += 1
        return v

    def short(self):
        self._clear()
        self._need(2)
        v = struct.unpack_from(">H", self.data, self.pos)[0]
        self.pos += 2
        return v

    def long(self):
        self._clear()
        self._need(4)
        v = struct.unpack_from(">I", self.data, self.pos)[0]
        self.pos += 4
        return v

    def longlong(self):
        self._clear()
        self._need(8)
        v = struct.unpack_from(">Q", self.data, self.pos)[0]
        self.pos += 8
        return v

    timestamp = longlong

    def shortstr(self):
        self._clear()
        self._need(1)
        n = self.data[self.pos]
        self.pos += 1
        self._need(n)
        b = bytes(self.data[self.pos:self.pos + n])
        self.pos += n
        return b.decode("utf-8", "surrogateescape")

    def longstr_bytes(self):
        self._clear()
        n = self.long()
        self._need(n)
        b = bytes(self.data[self.pos:self.pos + n])
        self.pos += n
        return b

    def longstr(self):
        b = self.longstr_bytes()
        try:
            return b.decode("utf-8")
        except UnicodeDecodeError:
            return b

    def table(self):
        self._clear()
        n = self.long()
        self._need(n)
        t = decode_table_body(self.data, self.pos, self.pos + n)
        self.pos += n
        return t


def _decode_value(r: Reader):
    tag = chr(r.octet())
    if tag == "S":
        return r.longstr()
    if tag == "x":
        return Typed("x", r.longstr_bytes())
    if tag == "I":
        r._need(4); v = struct.unpack_from(">i", r.data, r.pos)[0]; r.pos += 4; return v
    if tag == "l":
        r._need(8); v = struct.unpack_from(">q", r.data, r.pos)[0]; r.pos += 8; return Typed("l", v)
    if tag == "s":
        r._need(2); v = struct.unpack_from(">h", r.data, r.pos)[0]; r.pos += 2; return Typed("s", v)
    if tag == "b":
        r._need(1); v = struct.unpack_from(">b", r.data, r.pos)[0]; r.pos += 1; return Typed("b", v)
    if tag == "B":
        return Typed("B", r.octet())
    if tag == "u":
        return Typed("u", r.short())
    if tag == "i":
        return Typed("i", r.long())
    if tag == "t":
        return bool(r.octet())
    if tag == "d":
        r._need(8); v = struct.unpack_from(">d", r.data, r.pos)[0]; r.pos += 8; return v
    if tag == "f":
        r._need(4); v = struct.unpack_from(">f", r.data, r.pos)[0]; r.pos += 4; return Typed("f", v)
    if tag == "T":
        return Typed("T", r.longlong())
    if tag == "D":
        scale = r.octet()
        r._need(4); unscaled = struct.unpack_from(">i", r.data, r.pos)[0]; r.pos += 4
        return Decimal(unscaled).scaleb(-scale)
    if tag == "F":
        return r.table()
    if tag == "A":
        n = r.long()
        r._need(n)
        end = r.pos + n
        sub = Reader(r.data, r.pos, end)
        out = []
        while sub.pos < end:
            out.append(_decode_value(sub))
        r.pos = end
        return out
    if tag == "V":
        return None
    raise CodecError(f"unknown field tag {tag!r}", C.SYNTAX_ERROR)


def decode_table_body(data, start, end):
    r = Reader(data, start, end)
    out = {}
    while r.pos < end:
        k = r.shortstr()
        v = _decode_value(r)
        if k not in out:  # first duplicate wins (ValueReader.scala:71)
            out[k] = v
    return out


def decode_table(data) -> dict:
    r = Reader(data)
    return r.table()


# --------------------------------------------------------------------------- methods
class Method:
    """A decoded AMQP method: ``Method('basic.publish', exchange='x', ...)``."""

    __slots__ = ("spec", "args")

    def __init__(self, name_or_spec, **args):
        spec = BY_NAME[name_or_spec] if isinstance(name_or_spec, str) else name_or_spec
        self.spec = spec
        full = {}
        for fname, ftype in spec.fields:
            if fname in args:
                full[fname] = args.pop(fname)
            else:
                full[fname] = _DEFAULTS[ftype]
        if args:
            raise TypeError(f"unknown fields for {spec.name}: {sorted(args)}")
        self.args = full

    @property
    def name(self):
        return self.spec.name

    @property
    def class_id(self):
        return self.spec.class_id

    @property
    def method_id(self):
        return self.spec.method_id

    @property
    def has_content(self):
        return self.spec.content

    def __getattr__(self, k):
        try:
            return self.args[k]
        except KeyError:
            raise AttributeError(k) from None

    def __eq__(self, o):
        return isinstance(o, Method) and o.spec is self.spec and o.args == self.args

    def __repr__(self):
        return f"Method({self.spec.name!r}, {self.args!r})"

    def encode_payload(self) -> bytes:
        w = Writer()
        w.short(self.spec.class_id)
        w.short(self.spec.method_id)
        for fname, ftype in self.spec.fields:
            getattr(w, ftype)(self.args[fname])
        return w.getvalue()


_DEFAULTS = {"bit": False, "octet": 0, "short": 0, "long": 0, "longlong": 0, "shortstr": "",
             "longstr": b"", "table": {}, "timestamp": 0}


def decode_method(payload) -> Method:
    if len(payload) < 4:
        raise CodecError("method frame shorter than 4 bytes", C.FRAME_ERROR)
    cid, mid = struct.unpack_from(">HH", payload, 0)
    spec = BY_ID.get((cid, mid))
    if spec is None:
        raise CodecError(f"unknown class/method {cid}/{mid}", C.COMMAND_INVALID)
    r = Reader(payload, 4)
    args = {}
    for fname, ftype in spec.fields:
        if ftype == "longstr":
            args[fname] = r.longstr_bytes()
        else:
            args[fname] = getattr(r, ftype)()
    m = Method.__new__(Method)
    m.spec = spec
    m.args = args
    return m


# --------------------------------------------------------------------------- properties
def encode_properties(props: dict) -> bytes:
    """flags chain + property values (no class/weight/body-size)."""
    flags = []
    word = 0
    bit = 15
    vals = Writer()
    for i, (pname, ptype) in enumerate(BASIC_PROPERTIES):
        if bit == 0:  # continuation
            flags.append(word | 1)
            word = 0
            bit = 15
        present = props.get(pname) is not None
        if present:
            word |= 1 << bit
            getattr(vals, ptype)(props[pname])
        bit -= 1
    flags.append(word)
    return b"".join(struct.pack(">H", f) for f in flags) + vals.getvalue()


def decode_properties(data, pos=0, end=None):
    r = Reader(data, pos, end)
    presence = []
    while True:
        f = r.short()
        for b in range(15, 0, -1):
            presence.append(bool(f & (1 << b)))
        if not (f & 1):
            break
    props = {}
    for i, (pname, ptype) in enumerate(BASIC_PROPERTIES):
        if i < len(presence) and presence[i]:
            props[pname] = getattr(r, ptype)() if ptype != "longstr" else r.longstr_bytes()
    return props, r.pos


def encode_content_header(class_id: int, body_size: int, props: dict) -> bytes:
    return struct.pack(">HHQ", class_id, 0, body_size) + encode_properties(props)


def decode_content_header(payload):
    if len(payload) < 14:
        raise CodecError("content header too short", C.FRAME_ERROR)
    cid, weight, size = struct.unpack_from(">HHQ", payload, 0)
    props, _ = decode_properties(payload, 12)
    return cid, size, props


# --------------------------------------------------------------------------- frames
def encode_frame(ftype: int, channel: int, payload: bytes) -> bytes:
    return struct.pack(">BHI", ftype, channel, len(payload)) + payload + b"\xce"


def encode_method_frame(channel: int, method: Method) -> bytes:
    return encode_frame(C.FRAME_METHOD, channel, method.encode_payload())


def render_command(channel, method, props=None, body=b"", frame_max=131072) -> bytes:
    """Method + (header + body frames split at frame_max-8) (AMQCommand.scala:30-59)."""
    out = [encode_method_frame(channel, method)]
    if method.has_content:
        body = bytes(body)
        out.append(encode_frame(C.FRAME_HEADER, channel,
                                encode_content_header(method.class_id, len(body), props or {})))
        if body:
            step = (frame_max - C.FRAME_NON_BODY_SIZE) if frame_max else len(body)
            for i in range(0, len(body), step):
                out.append(encode_frame(C.FRAME_BODY, channel, body[i:i + step]))
    return b"".join(out)


class Frame:
    __slots__ = ("type", "channel", "payload")

    def __init__(self, ftype, channel, payload):
        self.type, self.channel, self.payload = ftype, channel, payload

    def __repr__(self):
        return f"Frame({self.type}, ch={self.channel}, {len(self.payload)}B)"

    def __eq__(self, o):
        return isinstance(o, Frame) and (o.type, o.channel, o.payload) == (self.type, self.channel, self.payload)


class FrameParser:
    """Incremental frame splitter with carry-over (FrameParser.scala:67-157)."""

    def __init__(self, frame_max=None):
        self.buf = bytearray()
        self.frame_max = frame_max

    def feed(self, data) -> list:
        self.buf += data
        out = []
        pos = 0
        buf = self.buf
        n = len(buf)
        while n - pos >= 7:
            ftype, ch, size = struct.unpack_from(">BHI", buf, pos)
            if self.frame_max and size + 8 > self.frame_max:
                raise CodecError(f"frame of {size} bytes exceeds frame-max", C.FRAME_ERROR)
            if n - pos < size + 8:
                break
            if buf[pos + 7 + size] != C.FRAME_END:
                raise CodecError("bad frame end marker", C.FRAME_ERROR)
            if ftype not in (1, 2, 3, 8):
                raise CodecError(f"bad frame type {ftype}", C.FRAME_ERROR)
            out.append(Frame(ftype, ch, bytes(buf[pos + 7:pos + 7 + size])))
            pos += size + 8
        del self.buf[:pos]
        return out


class Command:
    __slots__ = ("channel", "method", "props", "body", "raw_header")

    def __init__(self, channel, method, props=None, body=b"", raw_header=None):
        self.channel, self.method, self.props, self.body, self.raw_header = channel, method, props, body, raw_header

    def __repr__(self):
        return f"Command(ch={self.channel}, {self.method!r}, props={self.props}, body={len(self.body)}B)"


class CommandAssembler:
    """method -> [header -> body*] grouping (CommandAssembler.scala:33-130).

    Heartbeats come out as ``None`` commands on channel 0.
    """

    def __init__(self):
        self._pending = {}  # channel -> [method, props, raw_header, body_size, parts]

    def feed(self, frame: Frame):
        t = frame.type
        if t == C.FRAME_HEARTBEAT:
            return Command(0, None)
        ch = frame.channel
        if t == C.FRAME_METHOD:
            if ch in self._pending:
                raise CodecError("method frame while content pending", C.UNEXPECTED_FRAME)
            m = decode_method(frame.payload)
            if not m.has_content:
                return Command(ch, m)
            self._pending[ch] = [m, None, None, None, []]
            return None
        st = self._pending.get(ch)
        if st is None:
            raise CodecError("content frame without method", C.UNEXPECTED_FRAME)
        if t == C.FRAME_HEADER:
            if st[1] is not None:
                raise CodecError("duplicate content header", C.UNEXPECTED_FRAME)
            cid, size, props = decode_content_header(frame.payload)
            st[1], st[2], st[3] = props, bytes(frame.payload[12:]), size
            if size == 0:
                del self._pending[ch]
                return Command(ch, st[0], props, b"", st[2])
            return None
        if t == C.FRAME_BODY:
            if st[1] is None:
                raise CodecError("body frame before header", C.UNEXPECTED_FRAME)
            if not frame.payload:  # zero-length body frames are ignored (CommandAssembler.scala:101-105)
                return None
            st[4].append(frame.payload)
            got = sum(len(p) for p in st[4])
            if got > st[3]:
                raise CodecError("body larger than declared size", C.FRAME_ERROR)
            if got == st[3]:
                del self._pending[ch]
                return Command(ch, st[0], st[1], b"".join(st[4]), st[2])
            return None
        raise CodecError(f"bad frame type {t}", C.FRAME_ERROR)
