"""Two ranks of the sharded GPU server (golden planes, gloo) started by the launcher:
clients on different ranks declare, bind, publish and consume; messages cross ranks
through the per-step all-to-all; replicated ops are answered once applied everywhere."""

import json
import os
import time

import pytest

from chanamq_amd.client import ChannelClosed, Connection
from test_sharded_golden import _free_port

SMALL_CONF = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sharded_small.conf")

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(params=["golden", pytest.param("gpu", marks=pytest.mark.gpu)])
def cluster(request, tmp_path):
    from chanamq_amd.parallel.launch import Launcher
    env = dict(os.environ, PYTHONPATH=os.path.dirname(HERE))
    # 2 ranks share the one test GPU; the Python lockstep loop (remote consumers over the
    # Python link relay).  The pipelined front end: tests/test_gpu_sharded_server.py
    extra = ["--backend", "gloo", "--io", "native"] if request.param == "gpu" else []
    ln = Launcher(2, ["-m", "chanamq_amd.server.sharded", "--config", SMALL_CONF, "--plane", request.param, "--port", "0",
                      "--info-dir", str(tmp_path)] + extra, env=env).start()
    deadline = time.time() + 120
    while time.time() < deadline and not all((tmp_path / f"rank{r}.json").exists() for r in range(2)):
        assert not ln.poll(), f"rank exited early: {ln.poll()}"
        time.sleep(0.2)
    ports = [json.load(open(tmp_path / f"rank{r}.json"))["port"] for r in range(2)]
    yield ports
    ln.stop()


@pytest.mark.timeout(300)
def test_cross_rank_routing_and_replicated_topology(cluster):
    c0 = Connection(port=cluster[0], vhost="/")
    c1 = Connection(port=cluster[1], vhost="/")
    a = c0.channel()
    a.exchange_declare("sx", "topic")
    a.queue_declare("qa")
    a.queue_bind("qa", "sx", "a.*")
    b = c1.channel()
    b.exchange_declare("sx", "topic", passive=True)   # replicated to rank 1 already
    b.queue_declare("qb")
    b.queue_bind("qb", "sx", "*.b")
    a.basic_consume("qa", "ca", no_ack=True)
    b.basic_consume("qb", "cb", no_ack=True)
    p = c0.channel()
    for k in ("a.b", "a.x", "z.b"):
        p.basic_publish("sx", k, k.encode())
    assert [d.body for d in a.consume_n(2)] == [b"a.b", b"a.x"]
    assert [d.body for d in b.consume_n(2)] == [b"a.b", b"z.b"]
    # publishes from rank 1 reach rank 0's queue too
    p1 = c1.channel()
    p1.basic_publish("sx", "a.q", b"from-1")
    assert a.consume_n(1)[0].body == b"from-1"
    # a consumer on rank 1 of rank 0's queue (X2/X3 link): manual ack, nack-requeue
    p.basic_publish("sx", "a.r", b"r1")
    p.basic_publish("sx", "a.r", b"r2")
    assert [d.body for d in a.consume_n(2)] == [b"r1", b"r2"]
    a.basic_cancel("ca")
    r = c1.channel()
    r.basic_qos(prefetch_count=5)
    r.basic_consume("qa", "remote")
    c1.process(0.5)
    for i in range(8):
        p.basic_publish("sx", "a.z", b"z%d" % i)
    got = r.consume_n(5)
    assert [d.body for d in got] == [b"z%d" % i for i in range(5)]     # prefetch 5 across ranks
    r.basic_nack(got[1].delivery_tag, requeue=True)
    again = r.consume_n(1)[0]
    assert again.body == b"z1" and again.method.redelivered
    r.basic_ack(got[4].delivery_tag, multiple=True)
    rest = r.consume_n(3)
    assert [d.body for d in rest] == [b"z5", b"z6", b"z7"]
    r.basic_ack(rest[-1].delivery_tag, multiple=True)
    r.basic_ack(again.delivery_tag)
    r.basic_cancel("remote")
    c1.process(0.5)
    # everything was acked through the link: nothing comes back to a new consumer
    a.basic_consume("qa", "ca2", no_ack=True)
    p.basic_publish("sx", "a.end", b"end")
    assert a.consume_n(1)[0].body == b"end"
    # Basic.Get on rank 1 of rank 0's queue (pulled through a get link)
    a.basic_cancel("ca2")
    c0.process(0.3)
    for i in range(3):
        p.basic_publish("sx", "a.g", b"g%d" % i)
    c0.process(0.5)
    g = c1.channel()
    g0 = g.basic_get("qa")
    assert g0.body == b"g0" and g0.method.message_count == 2 and not g0.method.redelivered
    g1 = g.basic_get("qa", no_ack=True)
    assert g1.body == b"g1" and g1.method.delivery_tag == g0.method.delivery_tag + 1
    g.basic_nack(g0.method.delivery_tag, requeue=True)     # back at the head (of the get link)
    again = g.basic_get("qa")
    assert again.body == b"g0" and again.method.redelivered
    g.basic_ack(again.method.delivery_tag)
    assert g.basic_get("qa", no_ack=True).body == b"g2"
    assert g.basic_get("qa") is None
    c1.process(1.5)   # the idle get link closes; acks reached the owner: nothing comes back
    a.basic_consume("qa", "ca3", no_ack=True)
    p.basic_publish("sx", "a.end", b"end2")
    assert a.consume_n(1)[0].body == b"end2"
    c0.close()
    c1.close()


@pytest.mark.timeout(300)
def test_rank_death_durable_queue_reloaded(tmp_path):
    """HA at the protocol level: a client on rank 2 declares a durable queue there (queues
    live where they are declared) and publishes persistent messages with confirms; rank 2
    is killed; the survivor that inherits the queue reloads it from rank 2's store and a
    consumer on that rank receives every message."""
    from chanamq_amd.parallel.launch import Launcher
    env = dict(os.environ, PYTHONPATH=os.path.dirname(HERE))
    ln = Launcher(3, ["-m", "chanamq_amd.server.sharded", "--config", SMALL_CONF, "--plane", "golden", "--port", "0",
                      "--info-dir", str(tmp_path), "--store-dir", str(tmp_path / "store"), "--no-fsync"],
                  env=env).start()
    try:
        deadline = time.time() + 120
        while time.time() < deadline and not all((tmp_path / f"rank{r}.json").exists() for r in range(3)):
            assert not ln.poll(), f"rank exited early: {ln.poll()}"
            time.sleep(0.2)
        ports = [json.load(open(tmp_path / f"rank{r}.json"))["port"] for r in range(3)]
        c2 = Connection(port=ports[2], vhost="/")
        ch = c2.channel()
        ch.exchange_declare("hx", "direct", durable=True)
        ch.queue_declare("hq", durable=True)
        ch.queue_bind("hq", "hx", "k")
        ch.confirm_select()
        for i in range(20):
            ch.basic_publish("hx", "k", b"m%d" % i, {"delivery_mode": 2})
        assert ch.wait_for_confirms()
        ln.procs[2].kill()
        ln.procs[2].wait(30)
        got = None
        deadline = time.time() + 90
        while got is None and time.time() < deadline:
            for p in ports[:2]:
                c = Connection(port=p, vhost="/")
                try:
                    cc = c.channel()
                    cc.basic_consume("hq", "hc", no_ack=True)
                    got = [d.body for d in cc.consume_n(20, timeout=20)]
                    break
                except ChannelClosed:   # not (yet) the owner
                    pass
                finally:
                    c.close()
            if got is None:
                time.sleep(0.5)
        assert got == [b"m%d" % i for i in range(20)]
    finally:
        ln.stop()
