"""GPU correctness at bench scale (the paths bench.py's headline number actually takes):
1,024-slot connection tables and segment lists, 64 KB-per-producer TCP chunks split at
arbitrary offsets, multi-tile radix sorts, multi-block look-back scans, thousands of
deliveries per step.

* against the golden model for wide steps (256 producers x 16 topic queues, 64 producers x
  896 fan-out queues) at a size the Python golden can run: the same deliveries per step and
  consumer, contiguous tags, per-publisher order (cross-publisher interleaving within a
  step is unordered by design);
* at the full bench shape (config 2: 256 producers x 64 KB chunks per step), every
  delivery is decoded and checked: each message exactly once, per-(producer, queue) FIFO
  order, contiguous delivery tags per consumer channel, body checksums.
"""

import struct
from collections import defaultdict

import pytest

from chanamq_amd.engine.traffic import publish_command, split_stream
from chanamq_amd.protocol.codec import CommandAssembler, FrameParser

pytestmark = pytest.mark.gpu

VH = "AMQ.DEFAULT"
BENCH = dict(c_max=1024, chpc=4, q_max=2048, x_max=64, cons_max=2048, seg_max=1024, cmd_max=1 << 17,
             deliv_max=1 << 18, msg_max=1 << 20, ucap=4096, deliver_cap=8192, ingress_cap=40 << 20,
             egress_cap=192 << 20, log_bytes=2 << 30, log_block=4 << 20, ring_pool=1 << 22, tb_max=64,
             fan_max=1 << 20, carry_cap=256 << 10, dhash=4096, req_max=1 << 16)


def body_of(pid, seq, size):
    head = struct.pack(">II", pid, seq)
    fill = bytes(((pid * 131 + seq * 7 + k) & 0xFF) for k in range(16))
    return head + (fill * (size // 16 + 1))[:size - 8]


def producer_stream(pid, n, exchange, key_fn, size):
    return b"".join(publish_command(1, exchange, key_fn(pid, i), body_of(pid, i, size), {"delivery_mode": 1})
                    for i in range(n))


def setup(dp, producers, queues, kind):
    x = {"topic": "scale.topic", "fanout": "scale.fanout"}[kind]
    dp.declare_exchange(VH, x, kind)
    for q in range(queues):
        dp.declare_queue(VH, f"sq{q}", capacity=1 << 14 if queues <= 64 else 1 << 9)
        dp.bind(VH, f"sq{q}", x, f"scale.{q}.*" if kind == "topic" else "")
    for p in range(producers):
        dp.open_connection(p + 1, VH)
        dp.open_channel(p + 1, 1)
    cons = producers + 1
    for q in range(queues):
        dp.open_connection(cons + q, VH)
        dp.open_channel(cons + q, 1)
        dp.consume(cons + q, 1, VH, f"sq{q}", f"sc{q}", no_ack=True)
    return x, cons


def decode_all(buf):
    fp, ca = FrameParser(), CommandAssembler()
    out = []
    for fr in fp.feed(buf):
        c = ca.feed(fr)
        if c is not None:
            out.append(c)
    return out


def steps_for(streams, nsteps, seed):
    parts = {p: split_stream(s, nsteps, seed=seed + p) for p, s in streams.items()}
    return [{p: parts[p][k] for p in parts if k < len(parts[p])} for k in range(nsteps)]


@pytest.mark.parametrize("kind,producers,queues,per_prod", [("topic", 256, 16, 24), ("fanout", 64, 896, 6)])
def test_wide_step_matches_golden(gpu, kind, producers, queues, per_prod):
    from chanamq_amd.engine.dataplane import GpuDataPlane
    from chanamq_amd.engine.golden import GoldenDataPlane
    d = GpuDataPlane(**BENCH)
    g = GoldenDataPlane(c_max=BENCH["c_max"], chpc=BENCH["chpc"], q_max=BENCH["q_max"], x_max=BENCH["x_max"],
                        cons_max=BENCH["cons_max"], ucap=BENCH["ucap"], carry_cap=BENCH["carry_cap"],
                        deliver_cap=BENCH["deliver_cap"], ring_pool=BENCH["ring_pool"], deliv_max=BENCH["deliv_max"])
    outs = []
    for dp in (g, d):
        x, cons = setup(dp, producers, queues, kind)
        key = (lambda pid, i: f"scale.{(pid + i) % queues}.k") if kind == "topic" else (lambda pid, i: "any")
        streams = {p + 1: producer_stream(p, per_prod, x, key, 600) for p in range(producers)}
        res = []
        for k, inp in enumerate(steps_for(streams, 3, 11) + [{}]):
            r = dp.step(inp, now_ms=1_800_000_000_000 + k)
            res.append(r["egress"] if isinstance(r, dict) else r.egress)
        outs.append(res)
    # Commands of different connections that land in one step take their queue slots in
    # the order their segment blocks finish (one atomic per segment, k_frame_scan), so the
    # interleaving ACROSS publishers within a step is not fixed (AMQP orders per channel
    # only).  Compared exactly: per step and consumer the same deliveries (routing key,
    # properties, body), contiguous delivery tags, and per-publisher FIFO order.
    total = 0
    tags = {}
    for k, (a, b) in enumerate(zip(*outs)):
        assert sorted(a) == sorted(b), f"step {k}: egress connections differ"
        for c in a:
            ga, gb = decode_all(a[c]), decode_all(b[c])
            assert len(ga) == len(gb), f"step {k} conn {c}: delivery count"
            key = lambda cm: (cm.method.routing_key, cm.method.exchange, cm.method.consumer_tag, cm.body)  # noqa
            assert sorted(map(key, ga)) == sorted(map(key, gb)), f"step {k} conn {c}: deliveries differ"
            for cmds in (ga, gb):
                assert all(cm.method.name == "basic.deliver" for cm in cmds)
            for cmds, side in ((ga, 0), (gb, 1)):
                t0 = tags.get((side, c), 0)
                assert [cm.method.delivery_tag for cm in cmds] == list(range(t0 + 1, t0 + 1 + len(cmds)))
                tags[(side, c)] = t0 + len(cmds)
                last = {}
                for cm in cmds:
                    pid, seq = struct.unpack(">II", cm.body[:8])
                    assert seq > last.get(pid, -1), f"conn {c}: publisher {pid} out of order"
                    last[pid] = seq
            total += len(ga)
    assert total > 0


def test_bench_config2_shape_every_delivery_checked(gpu):
    """256 producers x ~64 KB per step (bench.py config 2), 4 steps + drain."""
    from chanamq_amd.engine.dataplane import GpuDataPlane
    producers, queues, size = 256, 16, 1024
    d = GpuDataPlane(**BENCH)
    x, cons = setup(d, producers, queues, "topic")
    per_step = 58                                    # ~64 KB of 1.1 KB messages per producer per step
    nsteps = 4
    n = per_step * nsteps
    key = lambda pid, i: f"scale.{(pid * 3 + i) % queues}.x{i % 10}"   # noqa: E731
    streams = {p + 1: producer_stream(p, n, x, key, size) for p in range(producers)}
    egress = defaultdict(bytearray)
    steps = [{p: s[k * len(s) // nsteps:(k + 1) * len(s) // nsteps] for p, s in streams.items()} for k in range(nsteps)]
    for k, inp in enumerate(steps + [{}, {}]):
        r = d.step(inp, now_ms=1_800_000_000_000 + k)
        for c, b in r.egress.items():
            egress[c] += b
        if k < nsteps:
            assert len(r.segs) >= producers and r.counters["n_pubs"] > 0
    c = d.last_counters
    assert c["n_ring_full"] == 0 and c["n_dropped_nomem"] == 0
    seen = set()
    for q in range(queues):
        cmds = decode_all(bytes(egress[cons + q]))
        tags = [cm.method.delivery_tag for cm in cmds]
        assert tags == list(range(1, len(cmds) + 1)), f"queue {q}: delivery tags not contiguous"
        last = {}
        for cm in cmds:
            assert cm.method.name == "basic.deliver" and cm.method.consumer_tag == f"sc{q}"
            assert not cm.method.redelivered
            pid, seq = struct.unpack(">II", cm.body[:8])
            assert cm.body == body_of(pid, seq, size), f"queue {q}: body of ({pid}, {seq}) corrupted"
            assert (pid * 3 + seq) % queues == q, "routed to the wrong queue"
            assert seq > last.get(pid, -1), f"queue {q}: producer {pid} out of order"
            last[pid] = seq
            assert (pid, seq) not in seen
            seen.add((pid, seq))
    assert len(seen) == producers * n
    # nothing leaked: every message released, the body log fully reclaimed
    assert c["n_live_msgs"] == 0 and c["live_bytes"] == 0
    assert c["log_head"] - c["log_tail"] <= BENCH["log_block"]


def test_closing_consumers_and_producers_leak_nothing(gpu):
    """Connections close mid-stream (consumers with deliveries in the step, producers with
    partial commands in their carry): every stored message is either delivered once or
    still queued, and live messages == queued messages."""
    from chanamq_amd.engine.dataplane import GpuDataPlane
    producers, queues, size = 32, 8, 1024
    d = GpuDataPlane(**BENCH)
    x, cons = setup(d, producers, queues, "topic")
    key = lambda pid, i: f"scale.{(pid + i) % queues}.k"   # noqa: E731
    streams = {p + 1: producer_stream(p, 400, x, key, size) for p in range(producers)}
    steps = steps_for(streams, 8, 21)
    delivered = set()
    for k, inp in enumerate(steps):
        r = d.step(inp, now_ms=1_800_000_000_000 + k)
        for q in range(queues):
            for cm in decode_all(r.egress.get(cons + q, b"")):
                key2 = struct.unpack(">II", cm.body[:8])
                assert key2 not in delivered
                delivered.add(key2)
        if k == 4:   # half the consumers and a quarter of the producers go away mid-stream
            for q in range(0, queues, 2):
                d.close_connection(cons + q)
            for p in range(0, producers, 4):
                d.close_connection(p + 1)
            steps = [{c: b for c, b in s.items() if c not in {p + 1 for p in range(0, producers, 4)}}
                     for s in steps]
    for k in range(3):
        d.step({}, now_ms=1_800_000_000_100 + k)
    c = d.last_counters
    queued = sum(d.message_count(d.queues[(VH, f"sq{q}")].slot) for q in range(queues))
    assert c["n_live_msgs"] == queued, (c["n_live_msgs"], queued)


def test_storm_redeliveries_flagged_and_complete(gpu):
    """Config 5 shape: manual-ack consumers; every 2nd step they nack-requeue everything
    outstanding, else ack everything.  Every message is eventually acked exactly once, and a
    message is flagged redelivered iff it was delivered before."""
    from chanamq_amd.engine.dataplane import GpuDataPlane
    from chanamq_amd.protocol.codec import Method, render_command
    producers, queues = 64, 64
    d = GpuDataPlane(**BENCH)
    d.declare_exchange(VH, "storm", "direct")
    for q in range(queues):
        d.declare_queue(VH, f"st{q}", capacity=1 << 12)
        d.bind(VH, f"st{q}", "storm", f"k{q}")
    for p in range(producers):
        d.open_connection(p + 1, VH)
        d.open_channel(p + 1, 1)
    cons = producers + 1
    for q in range(queues):
        d.open_connection(cons + q, VH)
        d.open_channel(cons + q, 1)
        d.qos(cons + q, 1, prefetch_count=64)
        d.consume(cons + q, 1, VH, f"st{q}", f"c{q}", no_ack=False)
    n = 40
    streams = {p + 1: producer_stream(p, n, "storm", lambda pid, i: f"k{(pid + i) % queues}", 200)
               for p in range(producers)}
    steps = steps_for(streams, 2, 5)
    delivered = defaultdict(int)
    ack = render_command(1, Method("basic.ack", delivery_tag=0, multiple=True))
    nack = render_command(1, Method("basic.nack", delivery_tag=0, multiple=True, requeue=True))
    for k in range(40):
        inp = dict(steps[k]) if k < len(steps) else {}
        if k >= 1:   # resolves every delivery of the earlier steps: nack-requeue storm, then acks
            ctl = nack if k % 2 == 0 and k < 8 else ack
            for q in range(queues):
                inp[cons + q] = ctl
        r = d.step(inp, now_ms=1_800_000_000_000 + k)
        ndel = 0
        for q in range(queues):
            for cm in decode_all(r.egress.get(cons + q, b"")):
                key = struct.unpack(">II", cm.body[:8])
                assert bool(cm.method.redelivered) == (delivered[key] > 0), f"redelivered flag of {key}"
                delivered[key] += 1
                ndel += 1
        if k >= 9 and ndel == 0:
            break
    assert len(delivered) == producers * n
    assert max(delivered.values()) >= 2                  # the storm really redelivered
    assert d.last_counters["n_live_msgs"] == 0           # every message acked and released
