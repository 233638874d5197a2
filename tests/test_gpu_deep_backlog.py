"""Deep backlog in HBM: one MI355X holds more than 100 GB of queued
1 KB message bodies -- a 128 GiB body log and a 2^27-entry message table, sized for the
288 GB of HBM3E -- with nobody consuming, then 16 consumers drain every message.  The
publishes are the headline bench's synthetic producer traffic (256 connections, 1 KB
bodies, topic exchange, 16 queues) pushed through the whole step (no TCP).  A sample of the
drained deliveries is decoded and checked body for body against what was published."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _check_bodies(egress, bodies, cap=2000):
    """Every delivery in a step's egress: a body some producer published, carried with the
    timestamp of a message that had that body (no body swapped, torn or stale)."""
    from chanamq_amd.protocol.codec import CommandAssembler, FrameParser
    n = 0
    for conn, data in egress.items():
        fp, ca = FrameParser(), CommandAssembler()
        for f in fp.feed(data):
            cmd = ca.feed(f)
            if cmd is None or cmd.method is None or cmd.method.name != "basic.deliver":
                continue
            j = bodies.get(cmd.body)
            assert j is not None, (conn, len(cmd.body), cmd.body[:16])
            assert (cmd.props["timestamp"] - 1_700_000_000) % 64 == j, (cmd.props, j)
            n += 1
            if n >= cap:
                return n
        assert not fp.buf, (conn, len(fp.buf))
    return n


@pytest.mark.timeout(600)
def test_hundred_gigabytes_of_1kb_bodies_then_drain(gpu):
    import bench
    from chanamq_amd.engine.dataplane import GpuDataPlane
    P, Q = 256, 16
    dp = GpuDataPlane(device=0, c_max=1024, chpc=4, q_max=64, cons_max=1024, seg_max=1024, cmd_max=1 << 17,
                      deliv_max=1 << 16, msg_max=1 << 27, ucap=4096, deliver_cap=8192, ingress_cap=32 << 20,
                      egress_cap=128 << 20, log_bytes=128 << 30, ring_pool=(Q << 23) + 4096, tb_max=64,
                      carry_cap=256 << 10)
    pool, segs, offs, blens, mps, wire, _ = bench.build_workload(dp, 0, P, Q, 1024, 65536, 8, cons_base=P,
                                                                 consume=False, qcap=1 << 23)
    base = pool.ctypes.data
    # the bodies every producer published (traffic.publish_stream: 64 random bodies per
    # producer, message i carries body i % 64 and timestamp 1_700_000_000 + i)
    bodies = {}
    for p in range(P):
        rows = np.random.default_rng(p).integers(0, 256, size=(64, 1024), dtype=np.uint8)
        for j in range(64):
            bodies[rows[j].tobytes()] = j
    target = 100 * 10**9
    slot = dp.info["log_bytes"]   # (for the message)
    published = steps = 0
    pending = []
    while True:
        b = steps % len(segs)
        pending.append(dp.submit_raw(segs[b], base + offs[b], blens[b]))
        steps += 1
        if len(pending) > 1:
            c = dp.finish(pending.pop(0), collect=False, wait_egress=False).counters
            published += c["n_pubs"]
            assert c["n_dropped_nomem"] == 0 and c["n_ring_full"] == 0, c
            if c["live_bytes"] >= target:
                break
        assert steps < 20000, (published, c["live_bytes"])
    for t in pending:
        c = dp.finish(t, collect=False).counters
        published += c["n_pubs"]
    live_msgs, live_bytes = c["n_live_msgs"], c["live_bytes"]
    assert live_bytes >= target and live_msgs == published, (live_bytes, live_msgs, published)
    assert sum(dp.message_count(q.slot) for q in dp.queue_by_slot.values() if q.name.startswith("bench.q")) == published
    # drain: 16 auto-ack consumers, empty steps until every queue is empty
    for i in range(Q):
        dp.consume(P + i, 1, "AMQ.DEFAULT", f"bench.q.0.{i}", f"drain-{i}", no_ack=True)
    empty = np.zeros(0, segs[0].dtype)
    delivered = checked = k = 0
    while delivered < published:
        sample = k % 37 == 0   # every 37th drain step: its deliveries' bodies against what was published
        r = dp.finish(dp.submit_raw(empty, 0, 0), collect=sample)
        c = r.counters
        delivered += c["n_deliv"]
        assert c["n_deliv"] > 0, (delivered, published)
        if sample:
            checked += _check_bodies(r.egress, bodies)
        k += 1
    assert checked >= 20000, checked
    c = dp.finish(dp.submit_raw(empty, 0, 0), collect=False).counters
    assert delivered == published and c["n_live_msgs"] == 0 and c["live_bytes"] == 0, (delivered, published, c)
