"""Body log of the GPU write-behind (csrc/core/bodylog.cpp): persistent message bytes go
from the step's record buffer to striped segment files (pwritev, CRC-framed), the WAL
keeps (segment, offset, length) rows written as one batched record per group commit
(Store::applyRows).  Recovery reads bodies back through select_message; a torn body reads
as absent (its message was never confirmed); segments whose rows are all gone are
unlinked.  Reference: CassandraOpService.scala:395-417 (insertMessage / insertQueueMsg)."""

import os

import numpy as np

from chanamq_amd.broker import load
from chanamq_amd.engine.layout import CONSUMED_REC, PERSIST_HDR


def _rec(mid, q, qpos, body, ex=b"x", rk=b"k", props=b"\x80\x00"):
    h = np.zeros(1, PERSIST_HDR)
    data = ex + rk + props + body
    pad = (-len(data)) % 8
    h["msg_id"], h["ts_ms"], h["qpos"], h["q"] = mid, 1234, qpos, q
    h["body_len"], h["props_len"], h["ex_len"], h["rk_len"] = len(body), len(props), len(ex), len(rk)
    h["size"] = PERSIST_HDR.itemsize + len(data) + pad
    return h.tobytes() + data + b"\0" * pad


def _consumed(items, kind):
    a = np.zeros(len(items), CONSUMED_REC)
    for i, (mid, q, pos) in enumerate(items):
        a[i] = (mid, pos, q, kind, (0, 0))
    return a.tobytes()


def _body(i, n=3000):
    return bytes([(i * 7 + k) % 251 for k in range(64)]) * (n // 64)


def _open(core, d, stripes=2, seg=1 << 20):
    st = core.Store()
    st.open(str(d), False)
    st.configure_body_log(stripes, seg)
    return st


def test_bodies_go_to_the_log_and_survive_reopen(tmp_path):
    core = load()
    st = _open(core, tmp_path / "s")
    for q in range(2):
        st.insert_queue_meta(f"v-_.dq{q}", -1, set(), True, 0)
    w = core.PersistWorker(st)
    for q in range(2):
        w.set_queue(q, f"v-_.dq{q}")
    w.start()
    buf = b"".join(_rec(100 + i, i % 2, i // 2, _body(i)) for i in range(400))
    w.submit(1, buf, b"")
    w.drain()
    w.stop()
    bs = st.body_stats()
    assert bs["records"] == 400 and bs["live_records"] == 400 and bs["segments"] >= 2, bs
    assert st.row_count("msgs") == 400 and st.row_count("queues") == 400
    # the WAL holds rows, not bodies
    assert os.path.getsize(tmp_path / "s" / "chanamq.wal") < 400 * 300
    m = st.select_message(137)
    assert m is not None and m[3] == _body(37) and m[4] == "x" and m[5] == "k" and m[7] == 1
    st.close()
    st2 = _open(core, tmp_path / "s")
    assert st2.row_count("msgs") == 400
    for i in (0, 199, 399):
        m = st2.select_message(100 + i)
        assert m is not None and m[3] == _body(i), i
        assert m[2][10:] == b"\x80\x00" and int.from_bytes(m[2][2:10], "big") == len(_body(i))
    _, rows, unacks = st2.select_queue("v-_.dq1")
    assert len(rows) == 200 and not unacks and rows[0] == (0, 101, len(_body(1)))
    st2.close()


def test_consumed_messages_free_their_segments(tmp_path):
    core = load()
    st = _open(core, tmp_path / "s", stripes=2, seg=1 << 20)
    st.insert_queue_meta("v-_.q", -1, set(), True, 0)
    w = core.PersistWorker(st)
    w.set_queue(0, "v-_.q")
    w.start()
    n = 2000                                        # ~6 MB of bodies: several 1 MB segments
    for s in range(10):
        ids = range(s * n // 10, (s + 1) * n // 10)
        w.submit(s + 1, b"".join(_rec(1000 + i, 0, i, _body(i)) for i in ids), b"")
        w.drain()
    before = st.body_stats()
    assert before["segments"] >= 4 and before["live_records"] == n, before
    items = [(1000 + i, 0, i) for i in range(n)]
    w.submit(20, b"", _consumed(items[:n // 2], 3))   # delivered, awaiting ack
    w.drain()
    _, rows, unacks = st.select_queue("v-_.q")
    assert len(rows) == n // 2 and len(unacks) == n // 2
    w.submit(21, b"", _consumed(items, 0))            # all acked
    w.drain()
    w.stop()
    after = st.body_stats()
    assert after["live_records"] == 0 and st.row_count("msgs") == 0
    assert after["reclaimed"] > 0 and after["segments"] <= 2, after   # only the stripes' current files
    st.close()
    left = os.listdir(tmp_path / "s" / "bodies")
    assert len(left) <= 2, left
    st2 = _open(core, tmp_path / "s")
    assert st2.row_count("msgs") == 0 and not os.listdir(tmp_path / "s" / "bodies")
    st2.close()


def test_torn_body_reads_as_absent_and_compaction_keeps_refs(tmp_path):
    core = load()
    st = _open(core, tmp_path / "s", stripes=1)
    st.insert_queue_meta("v-_.q", -1, set(), True, 0)
    w = core.PersistWorker(st)
    w.set_queue(0, "v-_.q")
    w.start()
    w.submit(1, b"".join(_rec(500 + i, 0, i, _body(i)) for i in range(8)), b"")
    w.drain()
    w.stop()
    st.compact()                                     # refs re-emitted as refs
    st.close()
    seg = sorted(os.listdir(tmp_path / "s" / "bodies"))
    assert len(seg) == 1
    path = tmp_path / "s" / "bodies" / seg[0]
    raw = bytearray(path.read_bytes())
    raw[-40] ^= 0xFF                                 # inside the last record's body
    path.write_bytes(bytes(raw))
    st2 = _open(core, tmp_path / "s", stripes=1)
    assert st2.row_count("msgs") == 8
    assert all(st2.select_message(500 + i)[3] == _body(i) for i in range(7))
    assert st2.select_message(507) is None
    assert st2.body_stats()["bad_reads"] == 1
    st2.close()


def test_memory_only_store_keeps_bodies_in_rows():
    core = load()
    st = core.Store()
    st.open("", False)
    assert not st.has_body_log()
    w = core.PersistWorker(st)
    w.set_queue(0, "v-_.q")
    w.start()
    w.submit(1, _rec(9, 0, 0, b"hello"), b"")
    w.drain()
    w.stop()
    assert st.select_message(9)[3] == b"hello"


def test_store_failure_is_reported_not_fatal(tmp_path):
    """a group commit whose body-log segment cannot be created (or whose pwritev /
    fdatasync failed: the error is sticky) throws on the PersistWorker thread.  The worker
    catches it: the process lives, drain() returns, nothing of the group (or later) is
    reported committed -- so no publisher confirm is released -- and stats() says why.
    Store.close() still closes its files."""
    core = load()
    st = _open(core, tmp_path / "s")
    st.insert_queue_meta("v-_.dq0", -1, set(), True, 0)
    # the bodies directory is a regular file: the first segment cannot be created
    (tmp_path / "s" / "bodies").write_bytes(b"not a directory")
    w = core.PersistWorker(st)
    w.set_queue(0, "v-_.dq0")
    w.start()
    w.submit(1, b"".join(_rec(100 + i, 0, i, _body(i)) for i in range(8)), b"")
    w.drain()
    w.submit(2, _rec(200, 0, 8, _body(1)), b"")   # after the failure: dropped, drain returns
    w.drain()
    s = w.stats()
    assert s["failed"] and "cannot create" in s["error"], s
    assert s["commits"] == 0
    w.stop()
    st.close()   # must not throw
