"""Packed persist records as the device writes them (k_persist_size / k_persist_pack): a
message's bytes ride its first record of the step only; its records for other durable
queues are 48-byte headers.  Both consumers of the buffer -- the native PersistWorker
(csrc/core/persist.cpp) and parse_persist (Python persistence) -- must store the full
message and one row per queue."""

import numpy as np

from chanamq_amd.broker import load
from chanamq_amd.engine.dataplane import parse_persist
from chanamq_amd.engine.layout import PERSIST_HDR


def _rec(mid, q, qpos, ex, rk, props, body, with_bytes):
    h = np.zeros(1, PERSIST_HDR)
    data = ex + rk + props + body
    pad = (-len(data)) % 8
    h["msg_id"], h["ts_ms"], h["qpos"], h["q"] = mid, 1234, qpos, q
    h["body_len"], h["props_len"], h["ex_len"], h["rk_len"] = len(body), len(props), len(ex), len(rk)
    h["size"] = PERSIST_HDR.itemsize + (len(data) + pad if with_bytes else 0)
    return h.tobytes() + (data + b"\0" * pad if with_bytes else b"")


def _buffer():
    # message 7 -> queues 0, 1, 2 with its bytes on the record for queue 1 (not the first
    # in the buffer); message 8 -> queue 0 only
    return (_rec(7, 0, 10, b"x", b"k", b"\x80\x00", b"B" * 100, False)
            + _rec(7, 1, 20, b"x", b"k", b"\x80\x00", b"B" * 100, True)
            + _rec(8, 0, 11, b"x", b"k2", b"", b"C" * 9, True)
            + _rec(7, 2, 30, b"x", b"k", b"\x80\x00", b"B" * 100, False))


def test_parse_persist_fills_header_only_records():
    recs = parse_persist(_buffer())
    assert [(r[0], r[2], r[3]) for r in recs] == [(7, 0, 10), (7, 1, 20), (8, 0, 11), (7, 2, 30)]
    for r in recs:
        if r[0] == 7:
            assert (r[5], r[6], r[7], r[8]) == (b"x", b"k", b"\x80\x00", b"B" * 100)
    assert recs[2][8] == b"C" * 9 and recs[2][6] == b"k2"


def test_native_worker_stores_message_once_with_a_row_per_queue(tmp_path):
    core = load()
    st = core.Store()
    st.open(str(tmp_path / "s"), False)
    w = core.PersistWorker(st)
    for q in range(3):
        w.set_queue(q, f"v-_.dq{q}")
    w.start()
    w.submit(1, _buffer(), b"")
    w.drain()
    w.stop()
    assert st.row_count("msgs") == 2
    assert st.row_count("queues") == 4
    m = st.select_message(7)
    assert m is not None and m[3] == b"B" * 100 and m[4] == "x" and m[5] == "k" and m[7] == 3
    st.close()
