"""HIP data plane vs golden model: byte-identical egress, control records, statuses."""

import pytest

from dp_scenarios import SCENARIOS, run

pytestmark = pytest.mark.gpu

from gpu_cfg import CFG  # noqa: E402


@pytest.fixture(params=[(True, 0), (False, 0), (True, 2), (True, 3)], ids=["graph", "eager", "copykernel", "hsa-sdma"])
def graph(request):
    return request.param


@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_gpu_matches_golden(gpu, name, graph):
    from chanamq_amd.engine.dataplane import GpuDataPlane
    from chanamq_amd.engine.golden import GoldenDataPlane

    g = GoldenDataPlane(c_max=CFG["c_max"], chpc=CFG["chpc"], q_max=CFG["q_max"], x_max=CFG["x_max"],
                        cons_max=CFG["cons_max"], ucap=CFG["ucap"], carry_cap=CFG["carry_cap"],
                        default_queue_capacity=CFG["default_queue_capacity"])
    d = GpuDataPlane(graph=graph[0], copy_engine=graph[1], **CFG)
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
