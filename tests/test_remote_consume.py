"""Remote consumption across ranks (parallel/links.py): a consumer on one
rank, its queue on another.  The per-connection byte stream a remote consumer receives
(over all steps) must equal what the same consumer receives from a single plane holding
everything — delivery tags, redelivered bits, exchange / routing key, properties,
bodies — including manual acks, nack-requeue and prefetch windows.  Links add one step
of latency, so streams are compared after the run, not step by step."""

import pytest

from chanamq_amd.engine.golden import GoldenDataPlane
from chanamq_amd.engine.traffic import ack_frame, publish_command
from chanamq_amd.protocol.codec import Method, render_command
from chanamq_amd.parallel.cluster import LocalCluster

VH = "AMQ.DEFAULT"


def golden(**kw):
    return GoldenDataPlane(default_queue_capacity=1 << 12, ring_pool=1 << 20, **kw)


def nack_frame(ch, tag, multiple=False, requeue=True):
    return render_command(ch, Method("basic.nack", delivery_tag=tag, multiple=multiple, requeue=requeue))


def pubs(n, key, seed, ch=1):
    return b"".join(publish_command(ch, "rx", key, b"%d-%d-" % (seed, i) + bytes(37 * (i % 5)),
                                    {"delivery_mode": 1, "message_id": "m%d" % i}) for i in range(n))


class Scenario:
    """queues: {name: owner rank}; producers: {conn: rank}; consumers: [(conn, rank, queue,
    tag, no_ack, prefetch)]; steps: [{conn: bytes}]"""

    def __init__(self, queues, producers, consumers, steps):
        self.queues, self.producers, self.consumers, self.steps = queues, producers, consumers, steps


def _topology(p):
    p.declare_exchange(VH, "rx", "direct")


def run_single(sc):
    p = golden()
    _topology(p)
    for q in sc.queues:
        p.declare_queue(VH, q)
        p.bind(VH, q, "rx", q)
    for c in list(sc.producers) + [c[0] for c in sc.consumers]:
        p.open_connection(c, VH)
        p.open_channel(c, 1)
    for c, _, q, tag, no_ack, pf in sc.consumers:
        if pf:
            p.qos(c, 1, pf)
        p.consume(c, 1, VH, q, tag, no_ack=no_ack)
    streams = {}
    for k, st in enumerate(sc.steps):
        for c, b in p.step(st, now_ms=1000 + k)["egress"].items():
            streams[c] = streams.get(c, b"") + b
    return streams


def run_cluster(sc, world, make=golden):
    cl = LocalCluster(lambda **kw: make(**kw), world)
    for p in cl.planes:
        _topology(p)
        for q, owner in sc.queues.items():
            p.shard_map.place(VH, q, owner % world)
            p.declare_queue(VH, q)
            p.bind(VH, q, "rx", q)
    rank_of = dict(sc.producers)
    rank_of.update({c[0]: c[1] % world for c in sc.consumers})
    for c, r in rank_of.items():
        cl[r % world].open_connection(c, VH)
        cl[r % world].open_channel(c, 1)
    for i, (c, r, q, tag, no_ack, pf) in enumerate(sc.consumers):
        p = cl[r % world]
        if pf:
            p.qos(c, 1, pf)
        if sc.queues[q] % world == r % world:
            p.consume(c, 1, VH, q, tag, no_ack=no_ack)
        else:   # remote: a link, then a local consumer of its shadow queue
            shadow = cl.link_open(100 + i, VH, q, r % world, pf)
            p.consume(c, 1, VH, shadow, tag, no_ack=no_ack)
    streams = {}
    for k, st in enumerate(sc.steps):
        split = [dict() for _ in range(world)]
        for c, b in st.items():
            split[rank_of[c] % world][c] = b
        for res in cl.step(split, now_ms=1000 + k):
            eg = res["egress"] if isinstance(res, dict) else res.egress
            for c, b in eg.items():
                streams[c] = streams.get(c, b"") + b
    return cl, streams


def sc_manual_ack_nack_requeue():
    # queue on rank 0, publisher on rank 0, consumer on rank 1 (prefetch 10, manual ack)
    steps = [{1: pubs(15, "rq", 0)}, {}, {}, {2: ack_frame(1, 5) + nack_frame(1, 7)}, {}, {}, {},
             {2: ack_frame(1, 16)}, {}, {}, {}, {2: ack_frame(1, 21)}, {}, {}]
    return Scenario({"rq": 0}, {1: 0}, [(2, 1, "rq", "rc", False, 10)], steps)


def sc_no_ack_from_every_rank():
    # publishers on every rank, queues on rank 0 and 1, no-ack consumers elsewhere
    steps = []
    for k in range(4):
        steps.append({1: pubs(6, "qa", 10 + k), 3: pubs(5, "qb", 20 + k), 4: pubs(4, "qa", 30 + k)})
    steps += [{}] * 4
    return Scenario({"qa": 0, "qb": 1}, {1: 0, 3: 1, 4: 2},
                    [(5, 1, "qa", "ca", True, 0), (6, 2, "qb", "cb", True, 0)], steps)


def sc_mixed_local_and_remote():
    # a local and a remote manual-ack consumer share one queue (round-robin at the owner)
    steps = [{1: pubs(12, "qm", 0)}, {}, {}, {2: ack_frame(1, 6), 3: ack_frame(1, 6)}, {}, {}, {},
             {2: ack_frame(1, 6), 3: ack_frame(1, 6)}, {}, {}]
    return Scenario({"qm": 0}, {1: 0}, [(2, 0, "qm", "local", False, 0), (3, 1, "qm", "remote", False, 0)],
                    steps)


SCENARIOS = {"manual_ack_nack_requeue": sc_manual_ack_nack_requeue, "no_ack_every_rank": sc_no_ack_from_every_rank}


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_remote_consumer_stream_matches_single_plane(name, world):
    sc = SCENARIOS[name]()
    single = run_single(sc)
    cl, clus = run_cluster(SCENARIOS[name](), world)
    for c, _, *_ in sc.consumers:
        assert c in single and single[c], c
        assert clus.get(c) == single[c], (c, len(clus.get(c, b"")), len(single[c]))
    # everything acked: no message left anywhere, links still open
    for p in cl.planes:
        assert p.memory_in_use() == 0


def test_mixed_local_and_remote_consumers_get_every_message_once():
    """Round-robin between a local and a remote consumer is not step-for-step the single
    plane's (the remote one's credit reaches the owner a step later), but every message is
    delivered exactly once across the two and all are acked."""
    import re
    sc = sc_mixed_local_and_remote()
    cl, clus = run_cluster(sc, 2)
    bodies = []
    for c in (2, 3):
        bodies += re.findall(rb"0-\d+-", clus.get(c, b""))
    assert sorted(bodies) == sorted(b"0-%d-" % i for i in range(12))
    assert all(p.memory_in_use() == 0 for p in cl.planes)


def test_link_close_returns_unacked_to_the_queue():
    """Cancel / channel close of a remote consumer: what it still held (in its shadow or
    unacked at the client) goes back to the owner's queue flagged redelivered."""
    sc = Scenario({"rq": 0}, {1: 0}, [(2, 1, "rq", "rc", False, 4)], [{1: pubs(10, "rq", 0)}, {}, {}])
    cl, clus = run_cluster(sc, 2)
    a, b = cl[0], cl[1]
    assert clus[2].count(b"\x00\x3c\x00\x3c") == 4           # prefetch 4 delivered on rank 1
    b.close_channel(2, 1)
    cl.link_close(100)
    for k in range(3):
        cl.step([{}, {}], now_ms=2000 + k)
    assert a.message_count(a.queues[(VH, "rq")].slot) == 10    # all back at the owner
    assert not cl.links[0].links and (VH, "amq.link.100") not in b.queues
    # a local consumer on the owner now gets them, the first four redelivered
    a.open_connection(7, VH)
    a.open_channel(7, 1)
    a.consume(7, 1, VH, "rq", "again", no_ack=True)
    eg = cl.step([{}, {}], now_ms=3000)[0]["egress"][7]
    assert eg.count(b"\x00\x3c\x00\x3c") == 10


def gpu_plane(**kw):
    import torch

    from chanamq_amd.engine.dataplane import GpuDataPlane
    from gpu_cfg import CFG
    torch.cuda.set_device(0)
    return GpuDataPlane(persist=1, **CFG, **kw)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_gpu_remote_consumer_stream_matches_single_plane(gpu, name, world):
    """LocalCluster of GPU planes (one device): the remote consumer's byte stream equals
    the single golden plane's."""
    from chanamq_amd.parallel.links import parse_delivers
    sc = SCENARIOS[name]()
    single = run_single(sc)
    cl, clus = run_cluster(SCENARIOS[name](), world, make=gpu_plane)
    for c, _, *_ in sc.consumers:
        if name == "manual_ack_nack_requeue":   # one publisher: byte-exact
            assert clus.get(c) == single[c], (c, len(clus.get(c, b"")), len(single[c]))
            continue
        # several publishers on one rank: their interleaving inside a step is not fixed
        # on the GPU, so compare tags, the multiset of messages and each publisher's order
        a, b = parse_delivers(single[c]), parse_delivers(clus.get(c, b""))
        assert [d[0] for d in b] == list(range(1, len(a) + 1))
        assert sorted(d[2:] for d in a) == sorted(d[2:] for d in b)
        for seed in {d[5].split(b"-")[0] for d in a}:
            assert [d[5] for d in a if d[5].split(b"-")[0] == seed] == \
                   [d[5] for d in b if d[5].split(b"-")[0] == seed]
    for p in cl.planes:
        assert p.memory_in_use() == 0


# ------------------------------------------------------------------ remote Basic.Get
def _get_setup(world, make=golden, n=5):
    """Queue ``rq`` on rank 0 holding ``n`` messages; connection 2 on the last rank."""
    sc = Scenario({"rq": 0}, {1: 0}, [], [{1: pubs(n, "rq", 0)}, {}])
    cl, _ = run_cluster(sc, world, make)
    b = world - 1
    cl[b].open_connection(2, VH)
    cl[b].open_channel(2, 1)
    shadow = cl.link_open(300, VH, "rq", b, get=True)
    return cl, b, shadow


def _remote_get(cl, b, shadow, pn, no_ack=False, now_ms=5000):
    """One pull, answered after a step; the answer is served from the shadow on rank b
    like the server does (parallel/links.py, server/gpu_broker.py _serve_gets)."""
    from chanamq_amd.parallel.links import set_get_ok_count
    assert cl.link_pull(300, pn) is True
    cl.step([{} for _ in cl.planes], now_ms=now_ms)
    got = cl.links[b].take_gets()
    assert [g[0] for g in got] == [pn]
    cl.links[b].before_step()   # restore the fetched message into the shadow
    _, _, cnt = got[0]
    if cnt is None:
        return None
    p = cl[b]
    frames, _ = p.basic_get(2, 1, p.queues[(VH, shadow)].slot, False)
    return set_get_ok_count(frames, cnt)


@pytest.mark.parametrize("world", [2, 3])
def test_remote_basic_get_matches_single_plane(world):
    """Basic.Get on rank b of a queue owned by rank 0: GetOk frames (tag, redelivered,
    exchange, routing key, remaining count, properties, body) equal a single plane's,
    the client's acks reach the owner, Get-Empty once drained."""
    single = golden()
    _topology(single)
    single.declare_queue(VH, "rq")
    single.bind(VH, "rq", "rx", "rq")
    for c in (1, 2):
        single.open_connection(c, VH)
        single.open_channel(c, 1)
    single.step({1: pubs(5, "rq", 0)}, now_ms=1000)
    want = [single.basic_get(2, 1, single.queues[(VH, "rq")].slot, False)[0] for _ in range(5)]

    cl, b, shadow = _get_setup(world)
    got = [_remote_get(cl, b, shadow, pn) for pn in range(1, 6)]
    assert got == want
    assert _remote_get(cl, b, shadow, 6) is None          # empty
    a = cl[0]
    assert a.message_count(a.queues[(VH, "rq")].slot) == 0
    # acks on rank b go back to the owner: every message released everywhere
    cl.step([{} if r != b else {2: ack_frame(1, 5, multiple=True)} for r in range(world)], now_ms=6000)
    for k in range(3):
        cl.step([{} for _ in range(world)], now_ms=6001 + k)
    assert all(p.memory_in_use() == 0 for p in cl.planes)


def test_remote_basic_get_unacked_returns_on_link_close():
    """A manual-ack Get never acked: closing the get link (idle close in the server)
    returns the message to the owner's queue, flagged redelivered."""
    cl, b, shadow = _get_setup(2, n=3)
    assert _remote_get(cl, b, shadow, 1) is not None
    cl[b].close_channel(2, 1)
    cl.link_close(300)
    for k in range(3):
        cl.step([{}, {}], now_ms=7000 + k)
    a = cl[0]
    assert a.message_count(a.queues[(VH, "rq")].slot) == 3
    frames, cnt = a.basic_get(1, 1, a.queues[(VH, "rq")].slot, True)
    assert frames[7 + 4 + 8] & 1 and cnt == 2           # redelivered, two left


@pytest.mark.gpu
def test_gpu_remote_basic_get_matches_golden(gpu):
    """GPU planes (LocalCluster on one device): the remote GetOk frames equal the golden
    cluster's, and acks release everything."""
    want = []
    cl, b, shadow = _get_setup(2)
    for pn in range(1, 4):
        want.append(_remote_get(cl, b, shadow, pn))
    gcl, gb, gshadow = _get_setup(2, make=gpu_plane)
    got = [_remote_get(gcl, gb, gshadow, pn) for pn in range(1, 4)]
    assert got == want and all(g is not None for g in got)
    gcl.step([{}, {2: ack_frame(1, 3, multiple=True)}], now_ms=6000)
    for k in range(3):
        gcl.step([{}, {}], now_ms=6001 + k)
    a = gcl[0]
    assert a.message_count(a.queues[(VH, "rq")].slot) == 2
