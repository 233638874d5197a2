"""Embedded Cassandra-schema store and broker restart recovery."""

import struct
import time

from chanamq_amd.broker import load
from chanamq_amd.client import Connection

TABLES = ("msgs", "queues", "queue_metas", "queue_unacks", "queues_deleted", "queue_metas_deleted",
          "queue_unacks_deleted", "exchanges", "binds", "vhosts")


def test_store_ops_and_replay(tmp_path):
    core = load()
    s = core.Store()
    s.open(str(tmp_path))
    hdr = struct.pack(">HQ", 0, 3) + b"\x10\x00\x02"   # weight | bodySize | flags(delivery mode) | 2
    s.insert_message(42, 1700000000000, hdr, b"abc", "ex", "rk", True, 2, 0)
    s.update_message_refer_count(42, 1)
    s.insert_queue_meta("AMQ.DEFAULT-_.q", -1, {"1-1-c"}, True, 0)
    for off in range(3):
        s.insert_queue_msg("AMQ.DEFAULT-_.q", off, 100 + off, 3, 0)
    s.consumed_queue_messages("AMQ.DEFAULT-_.q", 1, [(0, 100, 3), (1, 101, 3)])
    s.delete_queue_unack("AMQ.DEFAULT-_.q", 100)
    s.insert_exchange("AMQ.DEFAULT-_.ex", "direct", True, False, False, {"a": "b"})
    s.insert_bind("AMQ.DEFAULT-_.ex", "AMQ.DEFAULT-_.q", "rk", {})
    s.insert_vhost("v1", True)
    s.close()
    s2 = core.Store()
    s2.open(str(tmp_path))
    m = s2.select_message(42)
    assert m[2] == hdr and m[3] == b"abc" and m[7] == 1
    meta, msgs, unacks = s2.select_queue("AMQ.DEFAULT-_.q")
    assert meta[0] == 1 and meta[1] == {"1-1-c"}
    assert msgs == [(2, 102, 3)]            # rows after lconsumed only
    assert unacks == [(1, 101, 3)]          # correct (offset, msgid) columns: A.Q21 fixed
    x, binds = s2.select_exchange("AMQ.DEFAULT-_.ex")
    assert x[0] == "direct" and x[4] == {"a": "b"} and binds == [("AMQ.DEFAULT-_.q", "rk", {})]
    s2.pending_delete_queue("AMQ.DEFAULT-_.q")
    assert s2.row_count("queue_metas_deleted") == 1 and s2.row_count("queues_deleted") == 1
    assert s2.select_queue("AMQ.DEFAULT-_.q") is None
    for t in TABLES:
        s2.row_count(t)
    s2.compact()
    s2.close()
    s3 = core.Store()
    s3.open(str(tmp_path))
    assert s3.select_message(42) is not None and s3.select_vhost("v1") is True


def test_store_ttl_rows_expire(tmp_path):
    core = load()
    s = core.Store()
    s.open("")
    s.insert_message(7, 0, b"\x00" * 12, b"x", "", "q", True, 1, 50)
    assert s.select_message(7) is not None
    time.sleep(0.1)
    assert s.select_message(7) is None


def test_durable_messages_survive_restart(tmp_path):
    core = load()
    cfg = {"port": 0, "host": "127.0.0.1", "heartbeat": 0, "data_dir": str(tmp_path)}
    b = core.Broker(cfg)
    b.start()
    c = Connection(port=b.port)
    ch = c.channel()
    ch.exchange_declare("dx", "direct", durable=True)
    ch.queue_declare("dq", durable=True)
    ch.queue_declare("tq", durable=False)
    ch.queue_bind("dq", "dx", "k")
    ch.queue_bind("tq", "dx", "k")
    ch.confirm_select()
    for i in range(6):
        ch.basic_publish("dx", "k", b"p%d" % i, {"delivery_mode": 2 if i % 2 == 0 else 1})
    assert ch.wait_for_confirms()
    # take one persistent message unacked: it must come back (redelivered) after restart
    ch2 = c.channel()
    ch2.basic_qos(prefetch_count=1)
    ch2.basic_consume("dq", "hold")
    held = ch2.consume_n(1)[0]
    assert held.body == b"p0"
    c.sock.close()   # crash the client without acking
    time.sleep(0.1)
    b.stop()
    del b
    b2 = core.Broker(cfg)
    b2.start()
    c2 = Connection(port=b2.port)
    ch = c2.channel()
    ok = ch.queue_declare("dq", passive=True, durable=True)
    assert ok.message_count == 3           # persistent ones only (p0 requeued, p2, p4)
    ch.basic_consume("dq", "after", no_ack=True)
    got = ch.consume_n(3)
    assert sorted(d.body for d in got) == [b"p0", b"p2", b"p4"]
    # binding survived: route again
    ch.basic_publish("dx", "k", b"again", {"delivery_mode": 2})
    assert ch.consume_n(1)[0].body == b"again"
    c2.close()
    b2.stop()


def test_store_api_open_summary_and_rank_dirs(tmp_path):
    """chanamq_amd.store: open (nested directories created), table summary, per-rank dirs."""
    from chanamq_amd.store import open_store, rank_dir, summary
    d = rank_dir(str(tmp_path / "cluster"), 2)
    assert d.endswith("rank2")
    st = open_store(d, fsync=False)
    st.insert_queue_meta("AMQ.DEFAULT-_.q", -1, set(), True, 0)
    st.insert_message(7, 0, b"\0" * 10, b"body", "x", "k", True, 1, 0)
    st.insert_queue_msg("AMQ.DEFAULT-_.q", 0, 7, 4, 0)
    st.sync()
    st.close()
    st = open_store(d, fsync=False)
    s = summary(st)
    assert s["msgs"] == 1 and s["queues"] == 1 and s["queue_metas"] == 1
    st.close()


def test_round1_wal_replays_and_is_rewritten(tmp_path):
    """A WAL written before the CRC-32C format (no header, zlib CRC-32 records) is read
    and rewritten in the current format on open."""
    import struct
    import zlib

    from chanamq_amd.store import open_store
    d = tmp_path / "old"
    d.mkdir()
    recs = b""
    for name in ("AMQ.DEFAULT", "v2"):
        body = bytes([18]) + struct.pack(">I", len(name)) + name.encode() + b"\x01"   # OP_VH_INS
        recs += struct.pack(">I", len(body)) + body + struct.pack(">I", zlib.crc32(body))
    (d / "chanamq.wal").write_bytes(recs)
    st = open_store(str(d), fsync=False)
    assert sorted(st.vhost_ids()) == ["AMQ.DEFAULT", "v2"]
    st.close()
    assert (d / "chanamq.wal").read_bytes().startswith(b"CMQWAL2\n")
    st = open_store(str(d), fsync=False)
    assert sorted(st.vhost_ids()) == ["AMQ.DEFAULT", "v2"]
    st.close()
