"""Golden codec tests + C++/Python codec cross-checks."""

import random
import struct
from decimal import Decimal

import pytest

from chanamq_amd.protocol import constants as C
from chanamq_amd.protocol.codec import (CodecError, CommandAssembler, FrameParser, Method, Typed, Writer,
                                        decode_content_header, decode_method, decode_table,
                                        encode_content_header, encode_frame, encode_table, render_command)
from chanamq_amd.protocol.methods import BASIC_PROPERTIES, METHODS

TYPE_CODE = {"bit": 0, "octet": 1, "short": 2, "long": 3, "longlong": 4, "shortstr": 5, "longstr": 6,
             "table": 7, "timestamp": 8}


def sample_args(spec, rnd):
    out = {}
    for name, t in spec.fields:
        out[name] = {"bit": rnd.random() < 0.5, "octet": rnd.randrange(256), "short": rnd.randrange(65536),
                     "long": rnd.randrange(1 << 32), "longlong": rnd.randrange(1 << 64),
                     "shortstr": "s" * rnd.randrange(20), "longstr": bytes(rnd.randrange(256) for _ in range(7)),
                     "table": {"k": 1, "s": "v"}, "timestamp": rnd.randrange(1 << 40)}[t]
    return out


def test_every_method_roundtrips():
    rnd = random.Random(1)
    for spec in METHODS:
        m = Method(spec, **sample_args(spec, rnd))
        back = decode_method(m.encode_payload())
        assert back == m, spec.name


def test_bit_packing_lsb_first_and_flush():
    w = Writer()
    w.bit(True); w.bit(False); w.bit(True); w.short(7); w.bit(True)
    assert w.getvalue() == b"\x05\x00\x07\x01"


def test_field_table_tags_and_first_duplicate_wins():
    t = {"S": "str", "I": -5, "l": 1 << 40, "t": True, "d": 1.5, "D": Decimal("3.14"), "F": {"x": 1}, "A": [1, "a"],
         "V": None, "s": Typed("s", -2), "b": Typed("b", -1), "T": Typed("T", 99), "x": Typed("x", b"\x00\x01"),
         "f": Typed("f", 0.5)}
    enc = encode_table(t)
    dec = decode_table(enc)
    assert dec["S"] == "str" and dec["I"] == -5 and dec["t"] is True and dec["D"] == Decimal("3.14")
    assert dec["F"] == {"x": 1} and dec["A"] == [1, "a"] and dec["V"] is None
    # duplicate key: first wins (ValueReader.scala:71)
    body = b"\x01kI\x00\x00\x00\x01\x01kI\x00\x00\x00\x02"
    assert decode_table(struct.pack(">I", len(body)) + body) == {"k": 1}
    with pytest.raises(CodecError):
        decode_table(struct.pack(">I", 3) + b"\x01kZ")


def test_shortstr_limit():
    w = Writer()
    with pytest.raises(CodecError):
        w.shortstr("x" * 256)


def test_properties_roundtrip_and_flags():
    props = {"content_type": "text/plain", "headers": {"a": 1}, "delivery_mode": 2, "priority": 5,
             "expiration": "6000", "timestamp": 1700000000, "app_id": "x", "cluster_id": "c"}
    hdr = encode_content_header(60, 10, props)
    cid, size, back = decode_content_header(hdr)
    assert (cid, size) == (60, 10) and back == props
    assert len(BASIC_PROPERTIES) == 14
    flags = struct.unpack(">H", hdr[12:14])[0]
    assert flags & (1 << 15) and flags & (1 << 12) and not flags & 1


def test_heartbeat_frame_bytes():
    assert encode_frame(C.FRAME_HEARTBEAT, 0, b"") == bytes([8, 0, 0, 0, 0, 0, 0, 206]) == C.HEARTBEAT_FRAME


def test_body_split_at_frame_max_minus_8():
    m = Method("basic.publish", exchange="e", routing_key="k")
    raw = render_command(1, m, {}, b"x" * 10000, frame_max=4096)
    frames = FrameParser().feed(raw)
    bodies = [f for f in frames if f.type == C.FRAME_BODY]
    assert [len(f.payload) for f in bodies] == [4088, 4088, 1824]


@pytest.mark.parametrize("cut", [1, 5, 7, 8, 13, 40])
def test_parser_carry_over_every_offset(cut):
    raw = b"".join(render_command(1, Method("basic.publish", exchange="e", routing_key=f"k{i}"), {"priority": 1},
                                  bytes(range(i)), 4096) for i in range(30))
    p, a = FrameParser(), CommandAssembler()
    cmds = []
    for i in range(0, len(raw), cut):
        for f in p.feed(raw[i:i + cut]):
            c = a.feed(f)
            if c:
                cmds.append(c)
    assert [c.body for c in cmds] == [bytes(range(i)) for i in range(30)]


def test_zero_length_body_frames_ignored():
    m = Method("basic.publish", exchange="", routing_key="q")
    raw = (encode_frame(1, 1, m.encode_payload()) + encode_frame(2, 1, encode_content_header(60, 2, {}))
           + encode_frame(3, 1, b"") + encode_frame(3, 1, b"ab"))
    a = CommandAssembler()
    cmds = [c for c in (a.feed(f) for f in FrameParser().feed(raw)) if c]
    assert len(cmds) == 1 and cmds[0].body == b"ab"


def test_bad_end_marker_is_frame_error():
    with pytest.raises(CodecError) as e:
        FrameParser().feed(b"\x01\x00\x01\x00\x00\x00\x01x\x00")
    assert e.value.code == C.FRAME_ERROR


def test_cpp_method_table_matches_python():
    from chanamq_amd.broker import load
    table = load().method_table()
    assert len(table) == len(METHODS)
    for (cls, mid, name, fields, content), spec in zip(table, METHODS):
        assert (cls, mid, name, content) == (spec.class_id, spec.method_id, spec.name, spec.content)
        assert [(f, TYPE_CODE[t]) for f, t in spec.fields] == [tuple(x) for x in fields], name


def test_cpp_codec_reencodes_python_bytes_identically():
    from chanamq_amd.broker import load
    core = load()
    rnd = random.Random(2)
    for spec in METHODS:
        m = Method(spec, **sample_args(spec, rnd))
        if any(t == "table" for _, t in spec.fields):
            continue
        p = m.encode_payload()
        assert core.reencode_method(p) == p, spec.name
