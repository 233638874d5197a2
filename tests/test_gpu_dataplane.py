"""HIP data plane vs golden model: byte-identical egress, control records, statuses."""

import pytest

from dp_scenarios import SCENARIOS, run

pytestmark = pytest.mark.gpu

from gpu_cfg import CFG  # noqa: E402


# h2d-hsa: the ingress payload copies on an SDMA engine through HSA, waited for on the
# device by k_h2d_wait (single GPU without the overlapped ingest; bench --h2d-hsa), every
# payload over 8 KB split in halves over two SDMA engines (h2d_split_min lowered from 4 MB)
@pytest.fixture(params=[(True, 0), (False, 0), (True, 2), (True, 3), (True, 3, {"h2d_hsa": 1, "overlap": 0, "h2d_split": 1, "h2d_split_min": 4096})],
                ids=["graph", "eager", "copykernel", "hsa-sdma", "h2d-hsa"])
def graph(request):
    return request.param


@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_gpu_matches_golden(gpu, name, graph):
    from chanamq_amd.engine.dataplane import GpuDataPlane
    from chanamq_amd.engine.golden import GoldenDataPlane

    g = GoldenDataPlane(c_max=CFG["c_max"], chpc=CFG["chpc"], q_max=CFG["q_max"], x_max=CFG["x_max"],
                        cons_max=CFG["cons_max"], ucap=CFG["ucap"], carry_cap=CFG["carry_cap"],
                        default_queue_capacity=CFG["default_queue_capacity"])
    extra = graph[2] if len(graph) > 2 else {}
    d = GpuDataPlane(graph=graph[0], copy_engine=graph[1], **extra, **CFG)
    if extra.get("h2d_hsa"):
        assert d.info["h2d_hsa_engine"] >= 0
    steps_g = SCENARIOS[name](g)
    steps_d = SCENARIOS[name](d)
    og = run(g, steps_g, now_step_ms=3000)
    od = run(d, steps_d, now_step_ms=3000)
    for k, (a, b) in enumerate(zip(og, od)):
        assert a["segs"] == b["segs"], f"step {k} segs"
        assert a["ctrl"] == b["ctrl"], f"step {k} ctrl"
        assert a["events"] == b["events"], f"step {k} events"
        assert a["gets"] == b["gets"], f"step {k} basic.get"
        assert a["txbuf"] == b["txbuf"], f"step {k} tx-held commands"
        assert sorted(a["egress"]) == sorted(b["egress"]), f"step {k} egress conns"
        for c in a["egress"]:
            assert a["egress"][c] == b["egress"][c], f"step {k} conn {c} egress differs"


def test_engine_layout(gpu):
    from chanamq_amd.engine.dataplane import GpuDataPlane
    from chanamq_amd.engine.layout import STRUCT_SIZES

    d = GpuDataPlane(**CFG)
    sz = d.info["sizeof"]
    for k, v in STRUCT_SIZES.items():
        assert sz[k] == v, k


def test_topic_mfma_prefilter_exact(gpu):
    """Every (key, pattern) pair: MFMA prefilter + exact matcher == golden matcher."""
    import random

    from chanamq_amd.engine.dataplane import GpuDataPlane
    from chanamq_amd.engine.traffic import publish_stream
    from chanamq_amd.models.matcher import topic_match
    from chanamq_amd.protocol.codec import CommandAssembler, FrameParser

    rnd = random.Random(7)
    words = ["a", "b", "cc", "d", "*", "#"]
    pats = sorted({".".join(rnd.choice(words) for _ in range(rnd.randint(1, 5))) for _ in range(40)})
    keys = [".".join(rnd.choice(words[:4]) for _ in range(rnd.randint(1, 6))) for _ in range(200)]
    d = GpuDataPlane(**CFG)
    vh = "AMQ.DEFAULT"
    d.declare_exchange(vh, "t", "topic")
    for i, p in enumerate(pats):
        d.declare_queue(vh, f"q{i}")
        d.bind(vh, f"q{i}", "t", p)
        d.open_connection(10 + i, vh)
        d.open_channel(10 + i, 1)
        d.consume(10 + i, 1, vh, f"q{i}", f"c{i}", no_ack=True)
    d.open_connection(1, vh)
    d.open_channel(1, 1)
    s = publish_stream(len(keys), "t", lambda i: keys[i], 8, seed=1)
    r = d.step({1: s})
    for i, p in enumerate(pats):
        got = []
        fp, ca = FrameParser(), CommandAssembler()
        for fr in fp.feed(r.egress.get(10 + i, b"")):
            c = ca.feed(fr)
            if c is not None and c.method is not None:
                got.append(c.method.routing_key)
        want = [k for k in keys if topic_match(p, k)]
        assert got == want, p


def test_decode_windows_name_and_key_lengths(gpu):
    """k_decode reads exchange names (up to 31 bytes) and routing keys (up to 32) from
    32-byte register windows and takes the byte loops beyond: names and keys on both sides
    of those edges (trailing dots, empty words, more than 8 words) route exactly as the
    golden topic matcher and the direct bindings say."""
    from chanamq_amd.engine.dataplane import GpuDataPlane
    from chanamq_amd.engine.traffic import publish_stream
    from chanamq_amd.models.matcher import topic_match
    from chanamq_amd.protocol.codec import CommandAssembler, FrameParser

    keys = ["", "zz", "a..zz", "." * 32, "a" + "." * 31, ".".join("abcdefghijklmnop")]
    keys += ["a." + "b" * (n - 2) for n in (30, 31, 32, 33, 40)]
    keys += ["c" * (n - 3) + ".zz" for n in (32, 33)]
    k31, k32, k33 = keys[7], keys[8], keys[9]
    assert (len(k31), len(k32), len(k33)) == (31, 32, 33)
    pats = ["*", "*.*", "#", "a.#", "#.zz", k31, k32, k33]
    d = GpuDataPlane(**CFG)
    vh = "AMQ.DEFAULT"
    conn, want, stream = 10, {}, b""
    for n in (1, 30, 31, 32, 40):            # exchange name lengths
        x = "t" + "x" * (n - 1)
        d.declare_exchange(vh, x, "topic")
        for j, p in enumerate(pats):
            q = f"q{n}.{j}"
            d.declare_queue(vh, q)
            d.bind(vh, q, x, p)
            d.open_connection(conn, vh)
            d.open_channel(conn, 1)
            d.consume(conn, 1, vh, q, f"c{conn}", no_ack=True)
            want[conn] = [k for k in keys if topic_match(p, k)]
            conn += 1
        stream += publish_stream(len(keys), x, lambda i: keys[i], 8, seed=n)
    for n in (1, 40):                        # direct: the key hash from the window
        x = "d" + "y" * (n - 1)
        d.declare_exchange(vh, x, "direct")
        for k in (k31, k32, k33):
            q = f"dq{n}.{len(k)}"
            d.declare_queue(vh, q)
            d.bind(vh, q, x, k)
            d.open_connection(conn, vh)
            d.open_channel(conn, 1)
            d.consume(conn, 1, vh, q, f"c{conn}", no_ack=True)
            want[conn] = [k]
            conn += 1
        stream += publish_stream(len(keys), x, lambda i: keys[i], 8, seed=100 + n)
    d.open_connection(1, vh)
    d.open_channel(1, 1)
    r = d.step({1: stream})
    egress = r["egress"] if isinstance(r, dict) else r.egress
    for c, w in want.items():
        got = []
        fp, ca = FrameParser(), CommandAssembler()
        for fr in fp.feed(egress.get(c, b"")):
            cm = ca.feed(fr)
            if cm is not None and cm.method is not None:
                got.append(cm.method.routing_key)
        assert got == w, (c, w)


def _deliveries(raw):
    from chanamq_amd.protocol.codec import CommandAssembler, FrameParser
    fp, ca = FrameParser(), CommandAssembler()
    return [c for c in (ca.feed(f) for f in fp.feed(raw)) if c is not None and c.method.name == "basic.deliver"]


def test_egress_by_reference_window(gpu):
    """Egress by reference: deliveries of bodies that arrived in the same step are rendered
    without them (Counters.n_ref; the D2H is the frames + gather table) and spliced back on
    the host; a body whose ingress payload may have been recycled since (published earlier,
    delivered from the backlog) is rendered from HBM.  Both byte-exact after the gather."""
    from chanamq_amd.engine.dataplane import GpuDataPlane
    from chanamq_amd.engine.traffic import publish_stream

    d = GpuDataPlane(egress_ref=0, **CFG)
    vh = "AMQ.DEFAULT"
    d.declare_exchange(vh, "rx", "direct")
    d.declare_queue(vh, "rq", capacity=1024)
    d.bind(vh, "rq", "rx", "k")
    for c in (0, 1):
        d.open_connection(c, vh)
        d.open_channel(c, 1)
    # step 1: no consumer yet -- the bodies wait in HBM; the payload buffer is reused later
    r = d.step({0: publish_stream(6, "rx", lambda i: "k", 704, seed=1)})
    assert r.counters["n_deliv"] == 0
    d.step({0: b""})
    d.step({0: b""})   # (both payload buffers rewritten since step 1)
    d.consume(1, 1, vh, "rq", "c", no_ack=True)
    r = d.step({})
    got = _deliveries(r.egress.get(1, b""))
    assert len(got) == 6 and r.counters["n_ref"] == 0       # from HBM
    stream = publish_stream(6, "rx", lambda i: "k", 704, seed=2)
    r = d.step({0: stream})
    got2 = _deliveries(r.egress.get(1, b""))
    c = r.counters
    assert len(got2) == 6 and c["n_ref"] == 6 and c["ref_bytes"] == 6 * 704
    # the same step's bodies, byte-exact after the splice, and the D2H holds none of them
    from chanamq_amd.protocol.codec import CommandAssembler, FrameParser
    fp, ca = FrameParser(), CommandAssembler()
    pubs = [x for x in (ca.feed(f) for f in fp.feed(stream)) if x is not None]
    assert [g.body for g in got2] == [p.body for p in pubs]
    assert c["egress_bytes"] - 16 * c["n_deliv"] + c["ref_bytes"] >= 6 * 704
    assert c["egress_bytes"] < 6 * 704
    # off: every body rendered into HBM egress again
    d.eng.set_egress_ref(-1, 256)
    r = d.step({0: publish_stream(3, "rx", lambda i: "k", 704, seed=3)})
    assert r.counters["n_ref"] == 0 and len(_deliveries(r.egress.get(1, b""))) == 3


def test_lost_egress_gate_fails_within_deadline(gpu):
    """A gated egress copy whose gate is never opened (a step that died before its last
    kernel) surfaces as an engine error within the wait deadline instead of a host thread
    spinning forever; the engine still tears down."""
    import time

    from chanamq_amd.engine.dataplane import GpuDataPlane
    from chanamq_amd.engine.traffic import publish_stream

    d = GpuDataPlane(copy_engine=3, egress_gate=1, wait_timeout_ms=400, overlap=0, **CFG)
    if not d.info.get("egress_gate"):
        pytest.skip("engine built without gated egress")
    vh = "AMQ.DEFAULT"
    d.declare_exchange(vh, "gx", "fanout")
    d.declare_queue(vh, "gq", capacity=4096)
    d.bind(vh, "gq", "gx", "")
    for c in (0, 1):
        d.open_connection(c, vh)
        d.open_channel(c, 1)
    d.consume(1, 1, vh, "gq", "c", no_ack=True)
    for k in range(6):   # egress history: the next steps' D2H is queued at launch, gated
        assert d.step({0: publish_stream(20, "gx", lambda i: "", 512, seed=k)}).counters["n_deliv"] == 20
    d.eng.inject_gate_fault()
    t0 = time.monotonic()
    with pytest.raises(RuntimeError, match="did not complete"):
        d.step({0: publish_stream(20, "gx", lambda i: "", 512, seed=99)})
    assert time.monotonic() - t0 < 5.0
    assert d.eng.wait_failed()
    del d


def test_lost_ingress_copy_fails_loudly(gpu):
    """An HSA ingress copy the step's k_h2d_wait never sees complete (injected: the step
    polls a word no copy clears, with a short poll budget) fails that step's collection with
    an engine error instead of passing a stale ingress slot off as the step's bytes; the
    engine still tears down."""
    from chanamq_amd.engine.dataplane import GpuDataPlane
    from chanamq_amd.engine.traffic import publish_stream

    d = GpuDataPlane(copy_engine=3, overlap=0, h2d_hsa=1, **CFG)
    assert d.info["h2d_hsa_engine"] >= 0
    vh = "AMQ.DEFAULT"
    d.declare_exchange(vh, "hx", "fanout")
    d.declare_queue(vh, "hq", capacity=4096)
    d.bind(vh, "hq", "hx", "")
    for c in (0, 1):
        d.open_connection(c, vh)
        d.open_channel(c, 1)
    d.consume(1, 1, vh, "hq", "c", no_ack=True)
    for k in range(4):
        assert d.step({0: publish_stream(20, "hx", lambda i: "", 512, seed=k)}).counters["n_deliv"] == 20
    d.eng.inject_h2d_fault()
    with pytest.raises(RuntimeError, match="ingress copy of step"):
        d.step({0: publish_stream(20, "hx", lambda i: "", 512, seed=99)})
    assert d.eng.wait_failed()
    del d
