"""AMQP conversations against the GPU-data-path server (server/gpu_broker.py), with the
plane = golden model (CPU, always) and = HIP data plane (GPU box, marked gpu)."""

import pytest

from chanamq_amd.client import ChannelClosed, Connection, ConnectionClosed

SMALL = dict(c_max=64, chpc=8, q_max=64, x_max=64, cons_max=256, ucap=256, deliver_cap=4096)
GPU_CFG = dict(SMALL, seg_max=64, cmd_max=4096, deliv_max=4096, msg_max=1 << 14, ingress_cap=8 << 20,
               egress_cap=16 << 20, log_bytes=64 << 20, log_block=1 << 20, ring_pool=1 << 20, tb_max=64,
               carry_cap=1 << 18, dhash=1024, req_max=4096)


def _gpu_present():
    # HIP device count through the data-plane extension itself (torch's lazy CUDA init
    # reports no device once another library initialised HIP first in this process)
    from chanamq_amd import ops
    return ops.load().device_count() > 0


def make_plane(kind):
    if kind == "golden":
        from chanamq_amd.engine.golden import GoldenDataPlane
        return GoldenDataPlane(default_queue_capacity=1 << 12, ring_pool=1 << 20, **SMALL)
    if not _gpu_present():
        pytest.fail("GPU test scheduled on a machine without a GPU")
    from chanamq_amd.engine.dataplane import GpuDataPlane
    return GpuDataPlane(default_queue_capacity=1 << 12, **GPU_CFG)


@pytest.fixture(params=["golden-native", "golden-python", pytest.param("gpu-native", marks=pytest.mark.gpu),
                        pytest.param("gpu-python", marks=pytest.mark.gpu),
                        pytest.param("gpu-pipeline", marks=pytest.mark.gpu)])
def broker(request):
    from chanamq_amd.server.gpu_broker import GpuBroker
    kind, io = request.param.split("-")
    # (the pipeline front end sends every step's bodies by reference here, however small the
    # step: the production threshold, egress_ref_step_min, would leave these steps inline)
    b = GpuBroker(make_plane(kind), idle_step_ms=1.0, io=io, ingress_bytes=8 << 20,
                  fe_cfg={"egress_ref_step_min": 0} if io == "pipeline" else None).start()
    yield b
    b.stop()


def conn(b, **kw):
    return Connection(port=b.port, vhost="/", **kw)


def dump_state(b):
    """The pipelined server's control / stepper state (printed into a failing test's log)."""
    import time
    fe, lk = getattr(b, "fe", None), b.lock
    if fe is None or not hasattr(fe, "ctl_state"):
        return
    for k in range(2):
        print("ctl_state (held, first after, submitted, finished):", fe.ctl_state(), "steps", fe.stats()["steps"],
              "lock depth", lk.depth, "paused_at", lk.paused_at, "light", lk.light,
              "deltas", b.plane.eng.deltas_pending() if hasattr(b.plane, "eng") else None,
              "running", b._running, "ctl thread", [t.name for t in __import__("threading").enumerate()],
              "conns", {k2: v.state for k2, v in b.conns.items()})
        time.sleep(0.5)


def dump_on_channel_timeout(monkeypatch, b):
    """Every Connection.channel() of the test dumps the server state before it times out."""
    orig = Connection.channel

    def channel(self, *a, **kw):
        try:
            return orig(self, *a, **kw)
        except TimeoutError:
            dump_state(b)
            raise
    monkeypatch.setattr(Connection, "channel", channel)


def channel_or_dump(b, c):
    """c.channel(); on a timeout, the pipelined server's control / stepper state first."""
    try:
        return c.channel()
    except TimeoutError:
        dump_state(b)
        raise


def test_publish_consume_topic(broker):
    p = conn(broker)
    ch = p.channel()
    ch.exchange_declare("tx", "topic")
    for q, pat in (("qa", "a.*"), ("qb", "*.b"), ("qall", "#")):
        ch.queue_declare(q)
        ch.queue_bind(q, "tx", pat)
    c = conn(broker)
    cc = c.channel()
    for q in ("qa", "qb", "qall"):
        cc.basic_consume(q, "t-" + q, no_ack=True)
    keys = ["a.x", "y.b", "a.b", "zzz"]
    for i, k in enumerate(keys):
        ch.basic_publish("tx", k, f"m{i}".encode(), {"content_type": "text/plain"})
    got = cc.consume_n(1 + 1 + 4 + 2)   # a.x->qa,qall; y.b->qb,qall; a.b->all 3; zzz->qall
    by_tag = {}
    for d in got:
        by_tag.setdefault(d.method.consumer_tag, []).append(d.body)
    assert by_tag["t-qa"] == [b"m0", b"m2"]
    assert by_tag["t-qb"] == [b"m1", b"m2"]
    assert by_tag["t-qall"] == [b"m0", b"m1", b"m2", b"m3"]
    assert got[0].props.get("content_type") in ("text/plain", b"text/plain")
    p.close()
    c.close()


def test_default_exchange_and_declare_counts(broker):
    p = conn(broker)
    ch = p.channel()
    ok = ch.queue_declare("")          # server-named
    name = ok.queue
    assert name.startswith("tmp.")
    for i in range(5):
        ch.basic_publish("", name, b"x%d" % i)
    p.process(0.2)
    ok2 = ch.queue_declare(name, passive=True)
    assert ok2.message_count == 5 and ok2.consumer_count == 0
    assert ch.queue_purge(name) == 5
    p.process(0.1)
    assert ch.queue_declare(name, passive=True).message_count == 0
    ch.basic_publish("", name, b"after")
    p.process(0.1)
    assert ch.queue_delete(name) == 1
    with pytest.raises(ChannelClosed) as e:
        ch.queue_declare(name, passive=True)
    assert e.value.code == 404
    p.close()


def test_manual_ack_prefetch_and_redelivery(broker):
    p = conn(broker)
    ch = p.channel()
    ch.queue_declare("work")
    for i in range(10):
        ch.basic_publish("", "work", b"w%d" % i)
    c = conn(broker)
    cc = c.channel()
    cc.basic_qos(prefetch_count=3)
    cc.basic_consume("work", "wc")
    first = cc.consume_n(3)
    assert [d.body for d in first] == [b"w0", b"w1", b"w2"]
    c.process(0.2)
    assert len(cc.deliveries) == 0           # prefetch window full
    cc.basic_nack(first[1].delivery_tag, requeue=True)
    cc.basic_ack(first[2].delivery_tag)
    nxt = cc.consume_n(2)
    assert nxt[0].body == b"w1" and nxt[0].method.redelivered
    cc.basic_recover()
    again = cc.consume_n(3)
    assert sorted(d.body for d in again) == sorted([b"w0", nxt[0].body, nxt[1].body])
    assert all(d.method.redelivered for d in again)
    p.close()
    c.close()


def test_confirms_and_mandatory_return(broker):
    p = conn(broker)
    ch = p.channel()
    ch.exchange_declare("dx", "direct")
    ch.queue_declare("dq")
    ch.queue_bind("dq", "dx", "k")
    ch.confirm_select()
    ch.basic_publish("dx", "k", b"ok")
    ch.basic_publish("dx", "nokey", b"lost", mandatory=True)
    assert ch.wait_for_confirms()
    p._wait(lambda: ch.returns or None, ch)
    r = ch.returns[0]
    assert r.method.reply_code == 312 and r.body == b"lost"
    p.close()


def test_errors_unknown_exchange_and_unsupported(broker):
    p = conn(broker)
    ch = p.channel()
    ch.basic_publish("nope", "k", b"x")
    with pytest.raises(ChannelClosed) as e:
        p._wait(lambda: None, ch, timeout=3)
    assert e.value.code == 404
    ch2 = p.channel()
    ch2.queue_declare("g")
    with pytest.raises(ConnectionClosed) as e:    # 540 is a connection exception (AMQP 0-9-1)
        ch2.exchange_bind("amq.direct", "amq.fanout", "k")
    assert e.value.code == 540
    p.close()
    q = conn(broker)
    q.channel().queue_declare("g", passive=True)   # broker still serving
    q.close()


def test_basic_get_ack_nack_and_empty(broker):
    """Basic.Get on the data path (k_basic_get): GetOk carries the remaining count and the
    channel's delivery tags; manual-ack gets are acked / requeued like deliveries."""
    p = conn(broker)
    ch = p.channel()
    ch.queue_declare("gq")
    for i in range(4):
        ch.basic_publish("", "gq", f"g{i}".encode(), {"delivery_mode": 1})
    d0 = ch.basic_get("gq", no_ack=True)
    assert d0.body == b"g0" and d0.method.message_count == 3 and not d0.method.redelivered
    d1 = ch.basic_get("gq")
    assert d1.body == b"g1" and d1.method.message_count == 2
    assert d1.method.delivery_tag == d0.method.delivery_tag + 1
    ch.basic_ack(d1.method.delivery_tag)
    d2 = ch.basic_get("gq")
    assert d2.body == b"g2"
    ch.basic_nack(d2.method.delivery_tag, requeue=True)
    d2b = ch.basic_get("gq")
    assert d2b.body == b"g2" and d2b.method.redelivered
    ch.basic_reject(d2b.method.delivery_tag, requeue=False)
    d3 = ch.basic_get("gq", no_ack=True)
    assert d3.body == b"g3" and d3.method.message_count == 0
    assert ch.basic_get("gq") is None
    assert ch.queue_declare("gq", passive=True).message_count == 0
    # a consumer sees nothing left over from the gets
    c = conn(broker)
    cc = c.channel()
    cc.basic_consume("gq", "after", no_ack=True)
    ch.basic_publish("", "gq", b"tail")
    assert [d.body for d in cc.consume_n(1)] == [b"tail"]
    p.close()
    c.close()


def test_pipelined_basic_gets_answered_in_order(broker):
    """Many Basic.Gets in flight on one channel (served by the steps that decode them on
    the device planes): every message once, in queue order, then GetEmpty; a Get of an
    unnamed queue (the channel's last declared one) still works through the host."""
    p = conn(broker)
    ch = p.channel()
    ch.queue_declare("pg")
    for i in range(100):
        ch.basic_publish("", "pg", f"m{i:03d}".encode())
    ch.queue_declare("pg2")
    g = conn(broker)
    gch = g.channel()
    got, empty = [], 0
    for _ in range(3):
        ok, e = gch.basic_get_many("pg", 40, no_ack=True)
        got += ok
        empty += e
    assert [d.body for d in got] == [f"m{i:03d}".encode() for i in range(100)] and empty == 20
    assert [d.method.message_count for d in got[:3]] == [99, 98, 97]
    gch.queue_declare("pg2")
    ch.basic_publish("", "pg2", b"last")
    d = gch.basic_get("", no_ack=True)
    assert d is not None and d.body == b"last"
    p.close()
    g.close()


def test_basic_get_races_queue_delete(broker):
    """Basic.Gets racing a Queue.Delete on another connection: every Get is
    answered (GetOk / GetEmpty, or the channel closed 404 once the queue is gone) -- never
    resubmitted forever against the deleted slot -- and a queue declared right after the
    delete does not take over the deleted queue's slot (a Get staged for it cannot land
    there)."""
    import threading
    from chanamq_amd.client import ChannelClosed as CC
    a, b = conn(broker), conn(broker)
    ca, cb = a.channel(), b.channel()
    for r in range(3):
        name = f"race{r}"
        cb.queue_declare(name)
        for i in range(20):
            cb.basic_publish("", name, b"x%d" % i)
        b.process(0.1)
        answers, errs = [], []

        def getter():
            ch = ca
            try:
                for _ in range(60):
                    answers.append(ch.basic_get(name, no_ack=True))
            except CC as e:
                errs.append(e.code)
        old_slot = next(q.slot for k, q in broker.plane.queues.items() if k[1] == name)
        t = threading.Thread(target=getter)
        t.start()
        b.process(0.02)
        cb.queue_delete(name)
        cb.queue_declare(name + "-next")   # may not reuse the deleted slot
        assert next(q.slot for k, q in broker.plane.queues.items() if k[1] == name + "-next") != old_slot
        t.join(30)
        assert not t.is_alive(), "a Basic.Get was never answered"
        assert errs in ([], [404])
        if errs:
            ca = a.channel()
    with pytest.raises(ChannelClosed) as e:
        ca.basic_get("race0")
    assert e.value.code == 404
    a.close()
    b.close()


def test_transactions_commit_and_rollback(broker):
    """Tx on the data path: publishes and acks of a Tx channel take effect at Tx.Commit
    only (in order), Tx.Rollback drops them; a mandatory unroutable publish is returned
    at commit."""
    p = conn(broker)
    ch = p.channel()
    ch.queue_declare("txq")
    c = conn(broker)
    cc = c.channel()
    cc.basic_consume("txq", "tc", no_ack=True)
    ch.tx_select()
    for i in range(3):
        ch.basic_publish("", "txq", f"t{i}".encode())
    ch.basic_publish("", "no-such-queue", b"lost", mandatory=True)
    assert ch.queue_declare("txq", passive=True).message_count == 0
    ch.tx_commit()
    assert [d.body for d in cc.consume_n(3)] == [b"t0", b"t1", b"t2"]
    p._wait(lambda: (True,) if ch.returns else None, ch, timeout=5)
    assert ch.returns[0].method.reply_code == 312
    ch.basic_publish("", "txq", b"dropped")
    ch.tx_rollback()
    ch.basic_publish("", "txq", b"t3")
    ch.tx_commit()
    assert [d.body for d in cc.consume_n(1)] == [b"t3"]
    # acks are transactional too: a rolled-back ack leaves the message unacked
    cc.basic_cancel("tc")
    w = c.channel()
    w.basic_qos(prefetch_count=10)
    w.tx_select()
    ch.basic_publish("", "txq", b"a0")
    ch.basic_publish("", "txq", b"a1")
    ch.tx_commit()
    w.basic_consume("txq", "wc")
    got = w.consume_n(2)
    w.basic_ack(got[1].method.delivery_tag, multiple=True)
    w.tx_rollback()
    w.basic_recover(requeue=True)        # nothing was acked: both come back
    again = w.consume_n(2)
    assert [d.body for d in again] == [b"a0", b"a1"] and all(d.method.redelivered for d in again)
    w.basic_ack(again[1].method.delivery_tag, multiple=True)
    w.tx_commit()
    assert w.queue_declare("txq", passive=True).message_count == 0
    p.close()
    c.close()


@pytest.fixture(params=["golden", pytest.param("gpu", marks=pytest.mark.gpu),
                        pytest.param("gpu-pipeline", marks=pytest.mark.gpu)])
def wm_broker(request):
    from chanamq_amd.server.gpu_broker import GpuBroker
    kind, _, io = request.param.partition("-")
    b = GpuBroker(make_plane(kind), idle_step_ms=1.0, ingress_bytes=8 << 20, io=io or "native",
                  mem_high_watermark=40_000, mem_low_watermark=10_000).start()
    yield b
    b.stop()


def test_memory_watermark_blocks_and_unblocks(wm_broker):
    p = conn(wm_broker)
    ch = p.channel()
    ch.queue_declare("wm")
    for i in range(60):
        ch.basic_publish("", "wm", bytes(1000))
    p._wait(lambda: True if p.blocked else None, timeout=5)
    c = conn(wm_broker)
    cc = c.channel()
    cc.basic_consume("wm", "wmc", no_ack=True)
    assert len(cc.consume_n(60)) == 60
    p._wait(lambda: True if not p.blocked else None, timeout=5)
    # a client without the connection.blocked capability gets Channel.Flow instead
    q = conn(wm_broker, capabilities={"publisher_confirms": True})
    qc = q.channel()
    qc.queue_declare("wm2")            # no consumer: the bytes stay
    for i in range(60):
        qc.basic_publish("", "wm2", bytes(1000))
    q._wait(lambda: True if qc.flow_active is False else None, timeout=5)
    p.close(); c.close(); q.close()


def make_persist_plane(kind):
    if kind == "golden":
        from chanamq_amd.engine.golden import GoldenDataPlane
        return GoldenDataPlane(default_queue_capacity=1 << 12, ring_pool=1 << 20, persist=True, **SMALL)
    if not _gpu_present():
        pytest.fail("GPU test scheduled on a machine without a GPU")
    from chanamq_amd.engine.dataplane import GpuDataPlane
    return GpuDataPlane(default_queue_capacity=1 << 12, persist=1, persist_max=4096, persist_bytes=8 << 20,
                        restore_max=1024, restore_bytes=8 << 20, **GPU_CFG)


@pytest.mark.parametrize("kind", ["golden", pytest.param("gpu", marks=pytest.mark.gpu),
                                  pytest.param("gpu-pipeline", marks=pytest.mark.gpu)])
def test_durable_persistent_messages_survive_restart(kind, tmp_path):
    """Config 4 path: durable queue + delivery-mode 2 + confirms; restart recovers the
    unacked (redelivered first) and the unconsumed messages; non-persistent ones are gone."""
    from chanamq_amd.broker import load
    from chanamq_amd.server.gpu_broker import GpuBroker
    core = load()
    st = core.Store()
    st.open(str(tmp_path / "store"), True)
    kind, _, io = kind.partition("-")
    io = io or "native"
    b = GpuBroker(make_persist_plane(kind), idle_step_ms=1.0, ingress_bytes=8 << 20, store=st, io=io).start()
    p = conn(b)
    ch = p.channel()
    ch.exchange_declare("dur.x", "direct", durable=True)
    ch.queue_declare("dur.q", durable=True)
    ch.queue_bind("dur.q", "dur.x", "k")
    ch.confirm_select()
    for i in range(10):
        ch.basic_publish("dur.x", "k", b"p%d" % i, {"delivery_mode": 2})
    for i in range(3):
        ch.basic_publish("dur.x", "k", b"t%d" % i, {"delivery_mode": 1})
    assert ch.wait_for_confirms()
    assert st.row_count("msgs") == 10
    c = conn(b)
    cc = c.channel()
    cc.basic_qos(prefetch_count=4)
    cc.basic_consume("dur.q", "dc")
    got = cc.consume_n(4)
    assert [d.body for d in got] == [b"p0", b"p1", b"p2", b"p3"]
    cc.basic_ack(got[1].delivery_tag, multiple=True)     # p0, p1 consumed; p2, p3 stay unacked
    assert [d.body for d in cc.consume_n(2)] == [b"p4", b"p5"]   # the freed credit: unacked too
    import time
    end = time.time() + 5   # the acked rows go with the next group commit (persist-group-ms)
    while st.row_count("msgs") != 8 and time.time() < end:
        cc.connection.process(0.02) if hasattr(cc, "connection") else time.sleep(0.02)
    assert st.row_count("msgs") == 8
    b.stop()
    st.close()

    st2 = core.Store()
    st2.open(str(tmp_path / "store"), True)
    try:   # (what the store holds for the queue: in the failure message)
        from chanamq_amd.engine.control import normalize_vhost
        from chanamq_amd.engine.persistence import entity_id
        sel = st2.select_queue(entity_id(normalize_vhost("/"), "dur.q"))
        held = (sel[0], sorted(sel[1]), sorted(sel[2])) if sel is not None else None
    except Exception as e:   # noqa: BLE001
        held = repr(e)
    b2 = GpuBroker(make_persist_plane(kind), idle_step_ms=1.0, ingress_bytes=8 << 20, store=st2, io=io).start()
    assert b2.recovered == 8
    c2 = conn(b2)
    ch2 = c2.channel()
    ch2.basic_consume("dur.q", "dc2", no_ack=True)
    got2 = ch2.consume_n(8)
    assert [d.body for d in got2] == [b"p2", b"p3", b"p4", b"p5", b"p6", b"p7", b"p8", b"p9"]
    assert [bool(d.method.redelivered) for d in got2] == [True] * 4 + [False] * 4, held
    c2.process(0.3)
    assert st2.row_count("msgs") == 0                     # auto-acked: rows deleted
    # the durable topology came back too: publishing through the exchange still routes
    q2 = c2.channel()
    q2.basic_publish("dur.x", "k", b"again", {"delivery_mode": 2})
    assert ch2.consume_n(1)[0].body == b"again"
    c2.close()
    b2.stop()
    st2.close()


def test_admin_rest_on_gpu_server(broker):
    import json
    import urllib.request

    from chanamq_amd.server.admin import AdminServer
    adm = AdminServer(broker, 0).start()
    try:
        base = f"http://127.0.0.1:{adm.port}"
        assert urllib.request.urlopen(base + "/admin/vhost/put/vx").status == 200
        assert "vx" in broker.plane.vhosts
        p = conn(broker)
        ch = p.channel()
        ch.queue_declare("adm.q")
        ch.basic_publish("", "adm.q", b"x")
        p.process(0.2)
        qs = json.loads(urllib.request.urlopen(base + "/admin/queues").read())
        assert any(q["name"] == "adm.q" and q["ready"] == 1 for q in qs)
        st = json.loads(urllib.request.urlopen(base + "/admin/stats").read())
        assert st["connections_open"] >= 1
        p.close()
    finally:
        adm.stop()


def test_confirmed_publishes_into_a_small_queue_are_never_lost(broker):
    """A confirm-mode publisher fills a consumer-less queue declared with a 4,096-slot ring
    (GPU_CFG default) with 12,000 messages (within the 16,384-entry message table): the
    ring grows, so every publish is acked (none nacked) and every message is later
    delivered, in order."""
    n = 12000 if hasattr(broker.plane, "eng") else 5000   # the golden (CPU) plane is slow
    p = conn(broker)
    ch = p.channel()
    ch.queue_declare("deep")
    ch.confirm_select()
    for i in range(n):
        ch.basic_publish("", "deep", i.to_bytes(4, "big"))
        if i % 2000 == 1999:
            p.process(0.01)
    assert ch.wait_for_confirms(timeout=60)
    assert ch.queue_declare("deep", passive=True).message_count == n
    c = conn(broker)
    cc = channel_or_dump(broker, c)
    cc.basic_consume("deep", "deepc", no_ack=True)
    got = cc.consume_n(n, timeout=120)
    assert [int.from_bytes(d.body, "big") for d in got] == list(range(n))
    p.close()
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("io", ["native", "pipeline"])
def test_large_message_4mb_roundtrip(gpu, io):
    """A 4 MB message (32 body frames at frame-max 128 KB) is assembled on the device in
    a large per-connection carry, stored, routed and delivered intact (SURVEY §5.7;
    FrameParser.scala:67 has no size limit)."""
    from chanamq_amd.engine.dataplane import GpuDataPlane
    from chanamq_amd.server.gpu_broker import GpuBroker
    cfg = dict(GPU_CFG, carry_cap=8 << 20, egress_cap=64 << 20, log_bytes=256 << 20, log_block=16 << 20)
    b = GpuBroker(GpuDataPlane(default_queue_capacity=1 << 12, **cfg), idle_step_ms=1.0, io=io,
                  ingress_bytes=8 << 20).start()
    try:
        p = conn(b)
        ch = p.channel()
        ch.queue_declare("big")
        ch.confirm_select()
        body = bytes((i * 7 + 3) & 0xFF for i in range(4 << 20))
        ch.basic_publish("", "big", body)
        ch.basic_publish("", "big", b"small-after")
        assert ch.wait_for_confirms(timeout=30)
        c = conn(b)
        cc = c.channel()
        cc.basic_consume("big", "bigc", no_ack=True)
        got = cc.consume_n(2, timeout=30)
        assert len(got[0].body) == len(body) and got[0].body == body
        assert got[1].body == b"small-after"
        p.close()
        c.close()
    finally:
        b.stop()


@pytest.mark.gpu
def test_ttl_expired_bodies_freed_without_consumers_or_connections(gpu):
    """K12: messages with a per-message TTL in a queue nobody consumes are dropped at the
    queue head and their HBM freed, even after every connection is gone (the front end
    keeps sweeping while the device holds messages; MessageEntity.scala:168-198)."""
    import time
    from chanamq_amd.engine.dataplane import GpuDataPlane
    from chanamq_amd.server.gpu_broker import GpuBroker
    b = GpuBroker(GpuDataPlane(default_queue_capacity=1 << 12, **GPU_CFG), idle_step_ms=1.0, io="pipeline",
                  ingress_bytes=8 << 20).start()
    try:
        p = conn(b)
        ch = p.channel()
        ch.queue_declare("ttl.nobody")
        for i in range(200):
            ch.basic_publish("", "ttl.nobody", bytes(2000), {"expiration": "1500"})
        p.process(0.3)
        b._sync_fe_stats()
        assert b._fe_stats["live_bytes"] >= 200 * 2000
        p.close()
        end = time.time() + 10
        while time.time() < end:
            time.sleep(0.2)
            b._sync_fe_stats()
            if b._fe_stats["live_bytes"] == 0:
                break
        assert b._fe_stats["live_bytes"] == 0
    finally:
        b.stop()


@pytest.mark.gpu
def test_config5_storm_setup_64p64c_against_pipelined_server(gpu):
    """Regression (round-2 config-5 setup timeout): 64 producer and 64 consumer connections
    open, declare and attach against the pipelined server, then run a short Basic.Nack
    (requeue) storm under a memory watermark; setup must finish and traffic must flow both
    ways with no load-generator error."""
    import time
    from chanamq_amd.broker import load
    from chanamq_amd.engine.dataplane import GpuDataPlane
    from chanamq_amd.server.gpu_broker import GpuBroker
    plane = GpuDataPlane(c_max=512, chpc=8, q_max=256, cons_max=1024, seg_max=512, cmd_max=1 << 16,
                         deliv_max=1 << 16, msg_max=1 << 20, ucap=8192, deliver_cap=8192, ingress_cap=32 << 20,
                         egress_cap=96 << 20, log_bytes=1 << 30, ring_pool=1 << 23, tb_max=256,
                         default_queue_capacity=1 << 18, carry_cap=1 << 18)
    b = GpuBroker(plane, idle_step_ms=0.5, io="pipeline", io_threads=4, per_conn_read=128 << 10,
                  mem_high_watermark=256 << 20).start()
    try:
        t0 = time.time()
        r = load().run_load(dict(port=b.port, seconds=2.0, warmup=0.5, queue="c5.q", exchange="c5.x", threads=8,
                                 consumer_threads=4, producers=64, consumers=64, queues=16, msg_size=1024,
                                 auto_ack=False, prefetch=512, nack_every=2))
        wall = time.time() - t0
    finally:
        b.stop()
    assert r["error"] == "", r["error"]
    assert r["sent"] > 0 and r["received"] > 0
    assert wall < 60, f"64P x 64C setup + 2.5 s of load took {wall:.1f} s"


@pytest.mark.gpu
@pytest.mark.parametrize("io", ["native", "pipeline"])
def test_64mb_message_assembled_on_the_host(gpu, io):
    """A 64 MB publish (512 body frames, 256x the 256 KB connection carry) is handed to the
    host by the frame scan, assembled from the device carry + the socket, enqueued through
    the device's import path and delivered intact; its confirm comes from the device, the
    connection carries on with the publishes after it, a mandatory unroutable one comes
    back as Basic.Return, and one above the broker's limit closes the channel with 311
    (FrameParser.scala:67 has no size limit)."""
    from chanamq_amd.engine.dataplane import GpuDataPlane
    from chanamq_amd.server.gpu_broker import GpuBroker
    cfg = dict(GPU_CFG, egress_cap=192 << 20, log_bytes=512 << 20, log_block=32 << 20)
    plane = GpuDataPlane(default_queue_capacity=1 << 12, **cfg)
    b = GpuBroker(plane, idle_step_ms=1.0, io=io, ingress_bytes=8 << 20).start()
    try:
        assert plane.max_host_message() >= (64 << 20)
        p = conn(b)
        ch = p.channel()
        ch.queue_declare("huge")
        ch.confirm_select()
        body = bytes((i * 131 + 7) & 0xFF for i in range(256)) * ((64 << 20) // 256)
        ch.basic_publish("", "huge", b"before")
        ch.basic_publish("", "huge", body, {"delivery_mode": 1, "content_type": "application/octet-stream"})
        ch.basic_publish("", "huge", b"after")
        assert ch.wait_for_confirms(timeout=120)
        c = conn(b)
        cc = c.channel()
        cc.basic_consume("huge", "hc", no_ack=True)
        got = cc.consume_n(3, timeout=120)
        assert got[0].body == b"before" and got[2].body == b"after"
        assert len(got[1].body) == len(body) and got[1].body == body
        assert got[1].props.get("content_type") in ("application/octet-stream", b"application/octet-stream")
        # mandatory + unroutable: the host returns it
        ch.basic_publish("", "no.such.queue", body[:(1 << 20) * 3], mandatory=True)
        p._wait(lambda: ch.returns or None, ch, timeout=60)
        r = ch.returns[0]
        assert r.method.reply_code == 312 and r.body == body[:(1 << 20) * 3]
        # above the limit: the channel is closed with CONTENT_TOO_LARGE
        ch2 = p.channel()
        too_big = plane.max_host_message() + (1 << 20)
        with pytest.raises(Exception) as e:
            ch2.basic_publish("", "huge", bytes(too_big))
            ch2.queue_declare("huge", passive=True)
        assert "311" in str(e.value) or "CONTENT_TOO_LARGE" in str(e.value).upper()
        assert b.stats.get("big_publishes", 0) >= 2
        p.close()
        c.close()
    finally:
        b.stop()


@pytest.mark.gpu
@pytest.mark.parametrize("io", ["native", "pipeline"])
def test_cold_bodies_spill_to_host_memory_and_come_back(gpu, io):
    """A backlog three times the HBM body log: as the log fills, the broker moves the
    oldest queued bodies to the host spill ring (pinned host memory), the log tail
    advances and every publish is confirmed; the consumer then gets every message, in
    order and intact, the spilled ones rendered straight from host memory."""
    import time
    from chanamq_amd.engine.dataplane import GpuDataPlane
    from chanamq_amd.server.gpu_broker import GpuBroker
    cfg = dict(GPU_CFG, log_bytes=32 << 20, log_block=1 << 20, spill_bytes=256 << 20, msg_max=1 << 15)
    plane = GpuDataPlane(default_queue_capacity=1 << 14, **cfg)
    b = GpuBroker(plane, idle_step_ms=1.0, io=io, ingress_bytes=8 << 20, mem_high_watermark=0).start()
    try:
        p = conn(b)
        ch = p.channel()
        ch.queue_declare("cold")
        ch.confirm_select()
        n, size = 6144, 16 << 10   # 96 MB of bodies
        for k in range(n):
            ch.basic_publish("", "cold", k.to_bytes(4, "big") * (size // 4))
            if k % 64 == 63:
                assert ch.wait_for_confirms(timeout=60), f"publish {k} nacked (log full, no spill?)"
                time.sleep(0.002)
        assert ch.wait_for_confirms(timeout=60)
        assert b.stats.get("spilled_bytes", 0) > (32 << 20)
        assert plane.spill_used() > 0
        c = conn(b)
        cc = c.channel()
        cc.basic_qos(prefetch_count=512)
        cc.basic_consume("cold", "cc", no_ack=True)
        got = cc.consume_n(n, timeout=120)
        assert [int.from_bytes(d.body[:4], "big") for d in got] == list(range(n))
        assert all(d.body == d.body[:4] * (size // 4) for d in got[::97])
        p.close()
        c.close()
    finally:
        b.stop()


@pytest.mark.gpu
@pytest.mark.parametrize("io", ["native", "pipeline"])
def test_purge_of_more_durable_messages_than_persist_records_per_step(gpu, io, tmp_path):
    """A purge of a durable queue holding 3x persist_max persistent messages: the device's
    TTL skip takes at most a quarter of a step's store-record buffer and continues in the
    following steps, so every deletion reaches the store (no record buffer overflow, no
    rows left behind) and a restart recovers nothing (consumed > persist_max)."""
    import time
    from chanamq_amd.broker import load
    from chanamq_amd.server.gpu_broker import GpuBroker
    core = load()
    st = core.Store()
    st.open(str(tmp_path / "store"), True)
    b = GpuBroker(make_persist_plane("gpu"), idle_step_ms=1.0, ingress_bytes=8 << 20, store=st, io=io).start()
    try:
        p = conn(b)
        ch = p.channel()
        ch.queue_declare("deep.dur", durable=True)
        ch.confirm_select()
        n = 3 * 4096
        for i in range(n):
            ch.basic_publish("", "deep.dur", b"m%d" % i, {"delivery_mode": 2})
            if i % 1024 == 1023:
                assert ch.wait_for_confirms(timeout=60)
        assert ch.wait_for_confirms(timeout=60)
        assert st.row_count("msgs") == n
        assert ch.queue_purge("deep.dur") == n
        deadline = time.time() + 30
        while st.row_count("msgs") and time.time() < deadline:
            p.process(0.1)
        assert st.row_count("msgs") == 0
        p.close()
    finally:
        b.stop()
        st.close()
    st2 = core.Store()
    st2.open(str(tmp_path / "store"), True)
    b2 = GpuBroker(make_persist_plane("gpu"), idle_step_ms=1.0, ingress_bytes=8 << 20, store=st2, io=io).start()
    try:
        assert b2.recovered == 0
    finally:
        b2.stop()
        st2.close()


@pytest.mark.gpu
def test_manual_ack_durable_drain_past_record_budget(gpu, tmp_path):
    """one multiple Basic.Ack settling more durable persistent deliveries than a
    step's store-record budget (k_chan_advance's share of persist_max).  The device keeps
    the settles past the budget as slot marks and resolves them in the following steps,
    so the broker keeps running and every acked message leaves the store."""
    import time
    from chanamq_amd.broker import load
    from chanamq_amd.engine.dataplane import GpuDataPlane
    from chanamq_amd.server.gpu_broker import GpuBroker
    core = load()
    st = core.Store()
    st.open(str(tmp_path / "store"), True)
    cfg = dict(GPU_CFG, ucap=4096, deliv_max=256, persist_max=1024, cmd_max=1024)   # pair_max 4096
    plane = GpuDataPlane(default_queue_capacity=1 << 14, persist=1, persist_bytes=16 << 20, restore_max=1024,
                         restore_bytes=8 << 20, **cfg)
    pm = plane.info["persist_max"]
    budget = pm - 256 - (pm >> 2) - 64
    assert pm >= 2 * 256 + 4096 and budget < 4096     # one 4096-slot settle exceeds it
    b = GpuBroker(plane, idle_step_ms=1.0, ingress_bytes=8 << 20, store=st).start()
    try:
        p = conn(b)
        ch = p.channel()
        ch.queue_declare("drain.dur", durable=True)
        ch.confirm_select()
        n = 6000
        for i in range(n):
            ch.basic_publish("", "drain.dur", b"d%d" % i, {"delivery_mode": 2})
            if i % 1000 == 999:
                assert ch.wait_for_confirms(timeout=60)
        assert ch.wait_for_confirms(timeout=60)
        assert st.row_count("msgs") == n
        c = conn(b)
        cc = c.channel()
        cc.basic_consume("drain.dur", "drainer", no_ack=False)
        first = cc.consume_n(4096, timeout=60)
        assert len(first) == 4096
        cc.basic_ack(first[-1].delivery_tag, multiple=True)
        rest = cc.consume_n(n - 4096, timeout=60)
        assert [d.body for d in first + rest] == [b"d%d" % i for i in range(n)]
        cc.basic_ack(rest[-1].delivery_tag, multiple=True)
        deadline = time.time() + 30
        while st.row_count("msgs") and time.time() < deadline:
            c.process(0.1)
        assert st.row_count("msgs") == 0
        assert b._running
        p.close()
        c.close()
    finally:
        b.stop()
        st.close()


@pytest.mark.gpu
@pytest.mark.parametrize("io", ["native", "pipeline"])
def test_backlog_past_hbm_and_host_tiers_goes_to_the_cold_store(gpu, io, tmp_path):
    """A backlog 6x the HBM body log plus the host spill ring: the log spills to pinned
    host memory, the full ring moves cold bodies to the cold store on disk (third tier,
    MessageEntity.scala:174-186), publishers are never paused or nacked; the consumer then
    gets every message in order and intact -- each cold body read back into the ring
    just before its queue position is delivered.  With the native front end both tiers
    ride the steps: the stepper never pauses for them."""
    import time
    from chanamq_amd.engine.dataplane import GpuDataPlane
    from chanamq_amd.server.gpu_broker import GpuBroker
    cfg = dict(GPU_CFG, log_bytes=32 << 20, log_block=1 << 20, spill_bytes=64 << 20, msg_max=1 << 16)
    plane = GpuDataPlane(default_queue_capacity=1 << 14, **cfg)
    b = GpuBroker(plane, idle_step_ms=1.0, io=io, ingress_bytes=8 << 20, mem_high_watermark=0,
                  cold_dir=str(tmp_path / "cold"), cold_hot=2048, cold_window=1024).start()
    try:
        p = conn(b)
        ch = p.channel()
        ch.queue_declare("deep")
        ch.confirm_select()
        pauses0 = b.stats.get("pauses", 0)
        n, size = 36864, 16 << 10   # 576 MB of bodies: 6x (log + ring)
        for k in range(n):
            ch.basic_publish("", "deep", k.to_bytes(4, "big") * (size // 4))
            if k % 64 == 63:
                if not ch.wait_for_confirms(timeout=60):
                    b._sync_fe_stats()
                    fs = {x: (b._fe_stats or {}).get(x) for x in ("dropped_nomem", "ring_full", "log_used", "live_bytes",
                                                                  "spill_moved", "live_msgs")}
                    raise AssertionError(f"publish {k} nacked: {fs} {b.stats}")
                time.sleep(0.001)
        assert ch.wait_for_confirms(timeout=60)
        assert not b.blocked and b.stats.get("flow_off", 0) == 0
        assert b.stats.get("cold_out_bytes", 0) > (256 << 20), b.stats
        assert b.cold.bytes_on_disk() > (256 << 20)
        c = conn(b)
        cc = c.channel()
        cc.basic_qos(prefetch_count=512)
        cc.basic_consume("deep", "dc", no_ack=True)
        got = cc.consume_n(n, timeout=300)
        assert [int.from_bytes(d.body[:4], "big") for d in got] == list(range(n))
        assert all(d.body == d.body[:4] * (size // 4) for d in got[::101])
        assert b.stats.get("cold_in_bytes", 0) > (256 << 20)
        if io == "pipeline":   # (the consumer's own declare / consume are light sections)
            assert b.stats.get("cold_side_ops", 0) > 0 and b.stats.get("cold_errors", 0) == 0, b.stats
            assert b.stats.get("pauses", 0) - pauses0 <= 2, b.stats
        p.close()
        c.close()
    finally:
        b.stop()


@pytest.mark.gpu
def test_control_churn_rides_the_steps_without_a_drain(gpu, monkeypatch):
    """Connection open/close, channel open/close and consume/cancel while a publisher
    streams: handled in light control sections (their table writes staged and applied by
    the next step's first kernel, replies sent behind the deliveries in flight), so the
    stepper is never paused for them; a closed channel's unacked deliveries are still
    requeued before its slot is reused (its CloseOk waits for the step carrying the close,
    so the reopen rides a later one), and no delivery is lost."""
    import threading
    import time
    from chanamq_amd.engine.dataplane import GpuDataPlane
    from chanamq_amd.server.gpu_broker import GpuBroker
    b = GpuBroker(GpuDataPlane(default_queue_capacity=1 << 12, **GPU_CFG), idle_step_ms=1.0, io="pipeline",
                  ingress_bytes=8 << 20).start()
    dump_on_channel_timeout(monkeypatch, b)
    try:
        s = conn(b)
        sch = channel_or_dump(b, s)
        for q in ("load", "cq", "rq"):
            sch.queue_declare(q)
        for k in range(10):
            sch.basic_publish("", "rq", f"r{k}".encode())
        sink = conn(b)
        kch = channel_or_dump(b, sink)
        kch.basic_consume("load", "sink", no_ack=True)
        stop = threading.Event()
        sent = [0]

        def pump():
            pc = conn(b)
            pch = pc.channel()
            while not stop.is_set():
                for _ in range(50):
                    pch.basic_publish("", "load", sent[0].to_bytes(4, "big") * 64)
                    sent[0] += 1
                pc.process(0.002)
            pc.close()
        th = threading.Thread(target=pump, daemon=True)
        th.start()
        time.sleep(0.3)
        pauses0, light0 = b.stats.get("pauses", 0), b.stats.get("light_sections", 0)
        # manual-ack consumer takes the 10, its channel closes with them unacked
        rc = conn(b)
        r1 = rc.channel(5)   # (a fixed number: the reopen below reuses its device slot)
        r1.basic_consume("rq", "r", no_ack=False)
        try:
            first = r1.consume_n(10, timeout=20)
        except TimeoutError:
            print("r1 got", len(r1.deliveries), "stats", b.stats, "fe", b.fe.stats() if b.fe else None)
            dump_state(b)
            raise
        assert sorted(d.body for d in first) == sorted(f"r{k}".encode() for k in range(10))
        r1.close()
        r2 = rc.channel(5)   # same channel number (same device slot): gets them again, redelivered
        r2.basic_consume("rq", "r2", no_ack=False)
        again = r2.consume_n(10, timeout=20)
        assert sorted(d.body for d in again) == sorted(f"r{k}".encode() for k in range(10))
        assert all(d.method.redelivered for d in again)
        # consume / cancel and connection churn
        cc = conn(b)
        cch = cc.channel()
        for k in range(100):
            cch.basic_consume("cq", f"c{k}", no_ack=True)
            cch.basic_cancel(f"c{k}")
        for _ in range(20):
            x = conn(b)
            channel_or_dump(b, x)
            x.close()
        pauses1, light1 = b.stats.get("pauses", 0), b.stats.get("light_sections", 0)
        stop.set()
        th.join(20)
        # every publish arrives, in order
        got = kch.consume_n(sent[0], timeout=60)
        assert [int.from_bytes(d.body[:4], "big") for d in got] == list(range(sent[0]))
        assert light1 - light0 >= 150, (light0, light1)
        assert pauses1 == pauses0, (pauses0, pauses1, b.stats.get("pause_why"))
        for c_ in (s, sink, rc, cc):
            c_.close()
    finally:
        b.stop()


@pytest.mark.gpu
def test_consume_ok_precedes_first_delivery_in_light_sections(gpu):
    """Basic.Consume on a queue with a backlog while the steps keep running (a light control
    section): the consumer's rows ride a step, and the Basic.ConsumeOk is released behind
    that step's egress -- so the device must not dispatch to the new consumer in that same
    step (cons_active 2 -> 1 at the next step's k_stage), or a strict client (Java:
    "Unsolicited delivery") sees a Basic.Deliver for a tag it does not know yet."""
    import threading
    import time
    from chanamq_amd.engine.dataplane import GpuDataPlane
    from chanamq_amd.server.gpu_broker import GpuBroker
    b = GpuBroker(GpuDataPlane(default_queue_capacity=1 << 12, **GPU_CFG), idle_step_ms=1.0, io="pipeline",
                  ingress_bytes=8 << 20).start()
    try:
        s = conn(b)
        sch = s.channel()
        sch.queue_declare("load")
        names = [f"bq{k}" for k in range(12)]
        for q in names:
            sch.queue_declare(q)
            for i in range(40):
                sch.basic_publish("", q, f"{q}-{i}".encode())
        s.process(0.2)
        sink = conn(b)
        kch = sink.channel()
        kch.basic_consume("load", "sink", no_ack=True)
        stop = threading.Event()

        def pump():   # keeps the stepper busy: every consume below is handled beside the steps
            pc = conn(b)
            pch = pc.channel()
            while not stop.is_set():
                for _ in range(20):
                    pch.basic_publish("", "load", b"x" * 256)
                pc.process(0.002)
            pc.close()
        th = threading.Thread(target=pump, daemon=True)
        th.start()
        time.sleep(0.2)
        light0, pauses0 = b.stats.get("light_sections", 0), b.stats.get("pauses", 0)
        stricts = [conn(b, strict=True) for _ in range(3)]   # (chpc 8: channels per connection)
        for k, q in enumerate(names):
            ch = stricts[k % 3].channel()
            ch.basic_consume(q, f"t{k}", no_ack=(k % 2 == 0))
            got = ch.consume_n(40, timeout=20)
            assert sorted(d.body for d in got) == sorted(f"{q}-{i}".encode() for i in range(40))
        for sc in stricts:
            assert sc.violations == [], sc.violations[:3]
        assert b.stats.get("light_sections", 0) - light0 >= len(names)
        assert b.stats.get("pauses", 0) == pauses0, b.stats.get("pause_why")
        stop.set()
        th.join(20)
        for c_ in [s, sink] + stricts:
            c_.close()
    finally:
        b.stop()


@pytest.mark.gpu
@pytest.mark.timeout(180)
def test_store_failure_nacks_unconfirmed_publishes(gpu, tmp_path):
    """Config 4 into a store that fills up (a store quota: its writes then fail like a full
    disk): the write-behind reports the failure, every publish whose rows did not reach the
    disk gets Basic.Nack within about a second (they were held forever before), publishers
    are blocked, /admin/stats names the failure -- and every acked message is in the store."""
    import json
    import time

    from chanamq_amd.broker import load
    from chanamq_amd.server.gpu_broker import GpuBroker
    core = load()
    path = str(tmp_path / "store")
    st = core.Store()
    st.open(path, True)
    st.set_quota(3 << 20)
    b = GpuBroker(make_persist_plane("gpu"), idle_step_ms=1.0, ingress_bytes=8 << 20, store=st, io="pipeline").start()
    try:
        p = conn(b)
        ch = p.channel()
        ch.queue_declare("sq", durable=True)
        ch.confirm_select()
        body = b"s" * 4096
        sent, t_fail = 0, None
        while sent < 6000 and ch.flow_active and not p.blocked:
            for _ in range(25):
                ch.basic_publish("", "sq", body, {"delivery_mode": 2})
                sent += 1
            p.process(0.002)
            if t_fail is None and "store_failed" in b.stats:
                t_fail = time.monotonic()
        end = time.monotonic() + 20
        fate = {}

        def resolve():
            while ch.confirms:
                tag, multiple, ack = ch.confirms.popleft()
                for t in (range(1, tag + 1) if multiple else (tag,)):
                    fate.setdefault(t, ack)
            return len(fate) >= sent
        while not resolve() and time.monotonic() < end:
            p.process(0.01)
        t_done = time.monotonic()
        if t_fail is None:
            t_fail = t_done
        assert "store_failed" in b.stats, b.stats
        assert len(fate) >= sent, (len(fate), sent)
        acked = sorted(t for t in range(1, sent + 1) if fate[t])
        nacked = [t for t in range(1, sent + 1) if not fate[t]]
        assert nacked and acked, (len(acked), len(nacked))
        assert t_done - t_fail < 2.0, t_done - t_fail    # (stats are polled every 50 ms)
        assert b.stats.get("store_fail_nacks", 0) > 0 and b.blocked
        assert "No space left" in json.loads(b.stats_json())["store_failed"]
        p.close()
    finally:
        b.stop()
        st.close()
    st2 = core.Store()
    st2.open(path, True)   # every acked message is on disk
    assert st2.row_count("msgs") >= len(acked), (st2.row_count("msgs"), len(acked))
    st2.close()
