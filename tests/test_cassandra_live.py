"""Live Cassandra backend (chanamq_amd/store/cassandra_live.py): the store's change feed
written through to a keyspace while the broker runs, the keyspace always converging on the
store's rows, and a broker restarted from a store pulled back out of the keyspace.

No Cassandra here: the cluster is tests/cql_fake_server.py (CQL native protocol v4, its own
value codec from the reference schema, INSERT / DELETE by key / SELECT), so parity with a
real cluster stays unpinned."""

import os
import sys
import time

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from cql_fake_server import FakeCql  # noqa: E402

from chanamq_amd.store import open_store  # noqa: E402
from chanamq_amd.store.cassandra_live import CassandraMirror  # noqa: E402
from chanamq_amd.store.cql import ORDER, SCHEMA, rows  # noqa: E402


def _norm(v):
    if isinstance(v, (set, frozenset)):
        return repr(sorted(v))
    if isinstance(v, dict):
        return repr(sorted(v.items()))
    if isinstance(v, (bytes, bytearray, memoryview)):
        return bytes(v).hex()
    return repr(v)


def _same(srv, ks, st):
    """Every table of the keyspace holds exactly the store's live rows."""
    want = rows(st)
    for t in ORDER:
        got = list(srv.tables.get((ks, t), {}).values())

        def key(r):
            out = []
            for c, ty in SCHEMA[t][0]:
                v = r.get(c)
                if ty.startswith("set"):
                    v = set(v or ())
                elif ty.startswith("map"):
                    v = dict(v or {})
                out.append(_norm(v))
            return tuple(out)
        assert sorted(map(key, got)) == sorted(map(key, want[t])), (t, len(got), len(want[t]))


def test_mirror_converges_on_the_store_rows(tmp_path):
    srv = FakeCql()
    st = open_store(str(tmp_path / "s"), fsync=False)
    try:
        q, x = "AMQ.DEFAULT-_.q", "AMQ.DEFAULT-_.x"
        st.insert_vhost("AMQ.DEFAULT", True)
        st.insert_exchange(x, "topic", True, False, False, {})
        st.insert_queue_meta(q, -1, {"c1"}, True, 0)
        for i in range(4):   # rows before the mirror starts: its initial push carries them
            st.insert_message(100 + i, 1700000000000 + i, b"\0\0" + bytes(8), b"early%d" % i, "x", "a.b", True, 1, 0)
            st.insert_queue_msg(q, i, 100 + i, 6, 0)
        st.sync()
        m = CassandraMirror(st, port=srv.port, keyspace="live", interval_s=0.01, batch=16).start()
        _same(srv, "live", st)
        # changes while it runs: row inserts, single-row deletes, a range consume (partition
        # rewrite), unacks, binding churn, a message published and acked between two takes
        for i in range(4, 40):
            st.insert_message(100 + i, 1700000000000 + i, b"\0\0" + bytes(8), b"body%d" % i, "x", "a.b", True, 1, 0)
            st.insert_queue_msg(q, i, 100 + i, 5, 0)
        st.insert_bind(x, q, "a.*", {"k": "v"})
        st.insert_bind(x, q, "b.#", {})
        st.consumed_queue_messages(q, 9, [(8, 108, 5), (9, 109, 5)])   # 0..9 consumed, 8 and 9 unacked
        for i in range(8):
            st.delete_message(100 + i)
        st.delete_queue_msg(q, 20)
        st.delete_bind(x, q, "b.#")
        st.insert_queue_meta("AMQ.DEFAULT-_.q2", 3, set(), False, 0)
        st.insert_message(999, 1, b"\0\0" + bytes(8), b"gone", "x", "k", True, 1, 0)
        st.delete_message(999)
        st.sync()
        assert m.flush(10.0)
        _same(srv, "live", st)
        assert ("live", "msgs") in srv.tables and 999 not in {k[0] for k in srv.tables[("live", "msgs")]}
        # a queue deleted (rows moved to the *_deleted tables) and an exchange deleted
        st.delete_queue_unack(q, 108)
        st.pending_delete_queue(q)
        st.delete_exchange(x)
        st.sync()
        assert m.flush(10.0)
        _same(srv, "live", st)
        assert m.stats["errors"] == 0 and m.stats["deletes"] > 0 and m.stats["partitions"] > 0, m.stats
        m.stop()
    finally:
        st.close()
        srv.close()


def test_mirror_keeps_its_keys_through_a_cluster_outage(tmp_path):
    """A write that fails (cluster gone) is retried: nothing marked is lost, the keyspace
    converges once a cluster answers again."""
    srv = FakeCql()
    st = open_store(str(tmp_path / "s"), fsync=False)
    try:
        m = CassandraMirror(st, port=srv.port, keyspace="ks", interval_s=0.01).start()
        real = srv._run
        fail = [True]

        def flaky(cql, vals):
            if fail[0] and cql.startswith("INSERT INTO ks.msgs"):
                raise RuntimeError("node down")
            return real(cql, vals)
        srv._run = flaky
        for i in range(5):
            st.insert_message(i + 1, 1, b"\0\0" + bytes(8), b"m%d" % i, "x", "k", True, 1, 0)
        st.sync()
        time.sleep(0.3)
        assert m.stats["errors"] > 0
        fail[0] = False
        assert m.flush(10.0)
        _same(srv, "ks", st)
        m.stop()
    finally:
        st.close()
        srv.close()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("kind", ["golden", pytest.param("gpu-pipeline", marks=pytest.mark.gpu)])
def test_broker_writes_through_and_restarts_from_the_keyspace(tmp_path, kind):
    """Config 4 on the broker (store on disk; the golden data plane, or the HIP data plane
    behind the native front end, whose write-behind batches rows through Store.applyRows)
    with the live backend on:
    durable queue, persistent publishes with confirms, some consumed and acked.  The keyspace
    then holds exactly the store's rows; a fresh store pulled from it (what
    chana.mq.store.cassandra-recover does) starts a broker that recovers the unacked and the
    unconsumed messages."""
    from test_gpu_broker import conn, make_persist_plane

    from chanamq_amd.broker import load
    from chanamq_amd.server.gpu_broker import GpuBroker
    from chanamq_amd.store.cql_native import CqlClient, pull
    srv = FakeCql()
    core = load()
    st = core.Store()
    st.open(str(tmp_path / "store"), True)
    m = CassandraMirror(st, port=srv.port, keyspace="cmq", interval_s=0.01).start()
    plane, _, io = kind.partition("-")
    io = io or "native"
    b = GpuBroker(make_persist_plane(plane), idle_step_ms=1.0, ingress_bytes=8 << 20, store=st, io=io).start()
    try:
        p = conn(b)
        ch = p.channel()
        ch.exchange_declare("dur.x", "direct", durable=True)
        ch.queue_declare("dur.q", durable=True)
        ch.queue_bind("dur.q", "dur.x", "k")
        ch.confirm_select()
        for i in range(10):
            ch.basic_publish("dur.x", "k", b"p%d" % i, {"delivery_mode": 2})
        assert ch.wait_for_confirms()
        c = conn(b)
        cc = c.channel()
        cc.basic_qos(prefetch_count=4)
        cc.basic_consume("dur.q", "dc")
        got = cc.consume_n(4)
        cc.basic_ack(got[1].delivery_tag, multiple=True)   # p0, p1 acked; p2, p3 unacked
        end = time.time() + 5
        while st.row_count("msgs") != 8 and time.time() < end:
            c.process(0.02)
        assert st.row_count("msgs") == 8
        assert m.flush(10.0)
        _same(srv, "cmq", st)
        assert len(srv.tables[("cmq", "msgs")]) == 8 and len(srv.tables[("cmq", "exchanges")]) >= 1
    finally:
        b.stop()
        m.stop()
        st.close()
    st2 = core.Store()
    st2.open(str(tmp_path / "restored"), True)
    try:
        with CqlClient(port=srv.port) as cl:
            n = pull(cl, st2, keyspace="cmq")
        assert n["msgs"] == 8
        b2 = GpuBroker(make_persist_plane(plane), idle_step_ms=1.0, ingress_bytes=8 << 20, store=st2, io=io).start()
        try:
            assert b2.recovered == 8
            c2 = conn(b2)
            ch2 = c2.channel()
            ch2.basic_consume("dur.q", "dc2", no_ack=True)
            got2 = ch2.consume_n(8)
            assert sorted(d.body for d in got2) == [b"p%d" % i for i in range(2, 10)]
        finally:
            b2.stop()
    finally:
        st2.close()
        srv.close()
