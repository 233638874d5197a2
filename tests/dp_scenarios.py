"""Deterministic data-plane scenarios shared by the golden-model (CPU) tests and the
HIP-vs-golden (GPU) tests.  Each scenario is a function ``(dp) -> list[step inputs]``
that configures the control state and returns per-step ``{conn: bytes}`` inputs;
``unpause`` entries (``{'__unpause__': [conns]}``) are applied before the step.
"""

from chanamq_amd.engine.traffic import ack_frame, heartbeat, publish_command, publish_stream, split_stream
from chanamq_amd.protocol.codec import Method, encode_method_frame, render_command

VH = "AMQ.DEFAULT"


def sc_direct_split(dp):
    dp.declare_queue(VH, "q1")
    dp.declare_exchange(VH, "ex", "direct")
    dp.bind(VH, "q1", "ex", "k1")
    dp.open_connection(1, VH)
    dp.open_channel(1, 1)
    dp.open_connection(2, VH)
    dp.open_channel(2, 5)
    dp.consume(2, 5, VH, "q1", "c1", no_ack=True)
    s = publish_stream(40, "ex", lambda i: "k1" if i % 3 else "nokey", 300, seed=1)
    parts = split_stream(s, 4, seed=3)
    return [{1: p} for p in parts] + [{}]


def sc_default_exchange(dp):
    dp.declare_queue(VH, "orders")
    dp.open_connection(3, VH)
    dp.open_channel(3, 1)
    dp.consume(3, 1, VH, "orders", "amq.ctag-1", no_ack=True)
    dp.open_connection(4, VH)
    dp.open_channel(4, 2)
    s = publish_stream(10, "", lambda i: "orders", 50, channel=2, seed=2)
    return [{4: s}, {}]


def sc_topic(dp):
    dp.declare_exchange(VH, "tx", "topic")
    pats = {"qa": ["forex.*", "*.usd"], "qb": ["*.eur", "forex.*", "trade"], "qc": ["*"], "qd": ["quote.#"],
            "qe": ["#"], "qf": ["a.*.c.#.z"]}
    for q, ps in pats.items():
        dp.declare_queue(VH, q)
        for p in ps:
            dp.bind(VH, q, "tx", p)
    conn = 10
    for q in pats:
        dp.open_connection(conn, VH)
        dp.open_channel(conn, 1)
        dp.consume(conn, 1, VH, q, "t-" + q, no_ack=True)
        conn += 1
    dp.open_connection(1, VH)
    dp.open_channel(1, 7)
    keys = ["forex.eur", "forex", "trade.jpy", "forex.jpy", "trade", "quote", "quote.a.b", "x.usd",
            "a.b.c.z", "a.b.c.q.r.z", "a.b.c", "", "forex.", "a..b", "...", "w1.w2.w3.w4.w5.w6.w7.w8.w9"]
    s = publish_stream(len(keys) * 3, "tx", lambda i: keys[i % len(keys)], 64, channel=7, seed=4)
    return [{1: s}, {}]


def sc_fanout(dp):
    dp.declare_exchange(VH, "fx", "fanout")
    for i in range(3):
        dp.declare_queue(VH, f"f{i}")
        dp.bind(VH, f"f{i}", "fx", "")
        dp.open_connection(20 + i, VH)
        dp.open_channel(20 + i, 1)
        dp.consume(20 + i, 1, VH, f"f{i}", f"fc{i}", no_ack=True)
    dp.open_connection(1, VH)
    dp.open_channel(1, 1)
    s = publish_stream(25, "fx", lambda i: "any", 2000, seed=5, frame_max=4096)
    return [{1: s[:3000]}, {1: s[3000:]}, {}]


def sc_manual_ack(dp):
    dp.declare_queue(VH, "work")
    dp.open_connection(1, VH)
    dp.open_channel(1, 1)
    dp.open_connection(2, VH)
    dp.open_channel(2, 1)
    dp.qos(2, 1, prefetch_count=5)
    dp.consume(2, 1, VH, "work", "w", no_ack=False)
    s = publish_stream(12, "", lambda i: "work", 100, seed=6)
    return [{1: s}, {2: ack_frame(1, 3, multiple=True)}, {2: ack_frame(1, 5, multiple=False)},
            {2: ack_frame(1, 4, multiple=False)}, {2: ack_frame(1, 0, multiple=True)}, {}]


def sc_confirm_mandatory(dp):
    dp.declare_exchange(VH, "cx", "direct")
    dp.declare_queue(VH, "cq")
    dp.bind(VH, "cq", "cx", "ok")
    dp.open_connection(1, VH)
    dp.open_channel(1, 1)
    dp.confirm_select(1, 1)
    dp.open_connection(2, VH)
    dp.open_channel(2, 1)
    dp.consume(2, 1, VH, "cq", "cc", no_ack=True)
    parts = []
    for i in range(9):
        parts.append(publish_command(1, "cx", "ok" if i % 3 else "lost", bytes([i]) * 40,
                                     {"delivery_mode": 2}, mandatory=(i == 3)))
    return [{1: b"".join(parts)}, {}]


def sc_control_barrier(dp):
    dp.declare_queue(VH, "cb")
    dp.open_connection(1, VH)
    dp.open_channel(1, 1)
    dp.open_connection(2, VH)
    dp.open_channel(2, 1)
    dp.consume(2, 1, VH, "cb", "c", no_ack=True)
    a = publish_stream(3, "", lambda i: "cb", 30, seed=7)
    ctrl = encode_method_frame(1, Method("queue.declare", queue="other"))
    b = publish_stream(4, "", lambda i: "cb", 31, seed=8)
    return [{1: a + ctrl + b + heartbeat()}, {"__unpause__": [1]}, {}]


def sc_nack_requeue(dp):
    dp.declare_queue(VH, "nq")
    dp.open_connection(1, VH)
    dp.open_channel(1, 1)
    dp.open_connection(2, VH)
    dp.open_channel(2, 1)
    dp.qos(2, 1, prefetch_count=4)
    dp.consume(2, 1, VH, "nq", "n", no_ack=False)
    s = publish_stream(6, "", lambda i: "nq", 20, seed=9)
    nack = render_command(1, Method("basic.nack", delivery_tag=2, multiple=True, requeue=True))
    rej = render_command(1, Method("basic.reject", delivery_tag=3, requeue=False))
    return [{1: s}, {2: nack}, {}, {2: rej}, {}, {2: ack_frame(1, 0)}, {}]


def sc_ttl(dp):
    dp.declare_queue(VH, "tq", ttl_ms=1000)
    dp.open_connection(1, VH)
    dp.open_channel(1, 1)
    s1 = publish_stream(3, "", lambda i: "tq", 10, seed=10)
    s2 = b"".join(publish_command(1, "", "tq", b"x" * 10, {"expiration": "5000"}) for _ in range(2))
    return [{1: s1 + s2}, {}]


def sc_frame_error(dp):
    dp.declare_queue(VH, "eq")
    dp.open_connection(1, VH)
    dp.open_channel(1, 1)
    good = publish_stream(2, "", lambda i: "eq", 10, seed=11)
    bad = b"\x01\x00\x01\x00\x00\x00\x05hello\x00"  # wrong end marker
    return [{1: good + bad}]


def sc_basic_get(dp):
    dp.declare_queue(VH, "bg", ttl_ms=0)
    dp.open_connection(1, VH)
    dp.open_channel(1, 3)
    dp.open_connection(2, VH)
    dp.open_channel(2, 1)
    s = publish_stream(5, "", lambda i: "bg", 5000, channel=3, seed=12, frame_max=4096)
    s2 = publish_command(3, "", "bg", b"short-lived", {"expiration": "10"})
    return [{1: s + s2}, {"__get__": [(2, 1, "bg", True), (2, 1, "bg", False), (2, 1, "bg", False)]},
            {2: ack_frame(1, 2), "__get__": [(2, 1, "bg", False)]},
            {2: render_command(1, Method("basic.nack", delivery_tag=3, multiple=False, requeue=True))},
            {"__get__": [(2, 1, "bg", True), (2, 1, "bg", True), (2, 1, "bg", True), (2, 1, "bg", True)]},
            {2: ack_frame(1, 0, multiple=True)}, {}]


def get_cmd(ch, queue, no_ack):
    return render_command(ch, Method("basic.get", ticket=0, queue=queue, no_ack=no_ack))


def sc_wire_get(dp):
    """Basic.Get from the connection's bytes, served by the step itself: pipelined Gets of
    one (channel, queue, no-ack) in one step; a different Get or an ack after them waits
    for the next step (carry); GetEmpty on a drained queue; an unnamed queue, another
    connection's exclusive queue and a full delivery window go to the host."""
    dp.declare_queue(VH, "wg", ttl_ms=0)
    dp.declare_queue(VH, "wx", exclusive_owner=1)
    dp.open_connection(1, VH)
    dp.open_channel(1, 1)
    dp.open_connection(2, VH)
    dp.open_channel(2, 1)
    dp.open_channel(2, 2)
    pubs = publish_stream(7, "", lambda i: "wg", 700, seed=21)
    burst = (get_cmd(1, "wg", True) * 3 + get_cmd(1, "wg", False) * 2 + ack_frame(1, 5, multiple=True)
             + get_cmd(2, "wg", True))
    return [{1: pubs}, {2: burst}, {}, {}, {},
            {2: get_cmd(1, "wg", True) * 2},                        # 1 left: GetOk then GetEmpty
            {2: get_cmd(2, "wx", True)},                            # another connection's exclusive queue
            {"__unpause__": [2], 2: get_cmd(1, "", True)},          # unnamed: the host's
            {"__unpause__": [2]}]


def sc_tx_hold(dp):
    dp.declare_queue(VH, "txh")
    dp.open_connection(1, VH)
    dp.open_channel(1, 1)
    dp.open_channel(1, 2)
    dp.tx_select(1, 2)
    dp.open_connection(2, VH)
    dp.open_channel(2, 1)
    dp.consume(2, 1, VH, "txh", "c", no_ack=True)
    held = [publish_command(2, "", "txh", bytes([i]) * 40) for i in range(3)]
    live = [publish_command(1, "", "txh", bytes([9 - i]) * 41) for i in range(4)]
    ack = render_command(2, Method("basic.ack", delivery_tag=1, multiple=False))
    ctrl = encode_method_frame(2, Method("tx.commit"))
    s1 = held[0] + live[0] + held[1]
    s2 = held[2] + ack + live[1] + ctrl + live[2] + live[3]
    return [{1: s1[:70]}, {1: s1[70:] + s2[:50]}, {1: s2[50:]}, {"__unpause__": [1]}, {}]


def sc_window_wrap(dp):
    """Auto-ack deliveries over several steps total more than the channel's unacked window
    (ucap=256 in the test config): the window head must advance over several 64-slot waves
    per k_chan_advance pass or deliveries stall once the window wraps."""
    dp.declare_queue(VH, "wq")
    dp.open_connection(1, VH)
    dp.open_channel(1, 1)
    dp.open_connection(2, VH)
    dp.open_channel(2, 3)
    dp.consume(2, 3, VH, "wq", "wc", no_ack=True)
    return [{1: publish_stream(200, "", lambda i: "wq", 16, seed=10 + k)} for k in range(4)] + [{}]


def sc_confirm_ring_full(dp):
    """A confirm-mode publisher fills a 16-slot queue with no consumer: the step that
    overflows the ring confirms its range with Basic.Nack (never an Ack for a dropped
    message); later steps that store everything are acked again."""
    dp.declare_exchange(VH, "rx", "direct")
    dp.declare_queue(VH, "small", capacity=16, max_capacity=16)
    dp.declare_queue(VH, "big")
    dp.bind(VH, "small", "rx", "s")
    dp.bind(VH, "big", "rx", "b")
    dp.open_connection(1, VH)
    dp.open_channel(1, 1)
    dp.confirm_select(1, 1)
    dp.open_channel(1, 2)
    dp.confirm_select(1, 2)
    s1 = publish_stream(10, "rx", lambda i: "s", 32, seed=21)
    s2 = publish_stream(10, "rx", lambda i: "s", 32, seed=22)
    b2 = publish_stream(5, "rx", lambda i: "b", 32, channel=2, seed=23)
    s3 = publish_stream(3, "rx", lambda i: "b", 32, seed=24)
    return [{1: s1}, {1: s2 + b2}, {1: s3}, {}]


def sc_big_segment(dp):
    """One connection segment above 128 KB (the frame scan's re-validating path)."""
    dp.declare_queue(VH, "bs")
    dp.open_connection(1, VH)
    dp.open_channel(1, 1)
    dp.open_connection(2, VH)
    dp.open_channel(2, 1)
    dp.consume(2, 1, VH, "bs", "bsc", no_ack=True)
    s = publish_stream(150, "", lambda i: "bs", 1000, seed=25)
    assert len(s) > 128 << 10
    return [{1: s}, {}]


def sc_ring_growth(dp):
    """Queues grow: an 8-slot ring past half full doubles between steps, so a confirm-mode
    publisher's messages are all stored (acked) and later all delivered in order."""
    dp.declare_queue(VH, "grow", capacity=8)
    dp.open_connection(1, VH)
    dp.open_channel(1, 1)
    dp.confirm_select(1, 1)
    s = [publish_stream(n, "", lambda i: "grow", 24, seed=30 + k) for k, n in enumerate((6, 10, 15))]
    return [{1: s[0]}, {1: s[1]}, {1: s[2]}, {"__consume__": [(2, 1, "grow", "gc")]}, {}, {}]


def sc_mixed_multiple_settles(dp):
    """Several multiple-settles of both kinds on one channel in one step: each tag's fate
    is the first settle (wire order) that covers it (AMQChannel.scala:128-174), not
    "acks win" — a nack-requeue storm acks and nacks alternately within one step."""
    dp.declare_queue(VH, "mq")
    dp.open_connection(1, VH)
    dp.open_channel(1, 1)
    dp.open_connection(2, VH)
    dp.open_channel(2, 1)
    dp.qos(2, 1, prefetch_count=20)
    dp.consume(2, 1, VH, "mq", "m", no_ack=False)
    s = publish_stream(16, "", lambda i: "mq", 20, seed=40)

    def nack(tag, multiple=True, requeue=True):
        return render_command(1, Method("basic.nack", delivery_tag=tag, multiple=multiple, requeue=requeue))
    mixed = (nack(4) + ack_frame(1, 8, multiple=True) + nack(10, requeue=False) + ack_frame(1, 12, multiple=False)
             + nack(14))
    rev = ack_frame(1, 18, multiple=True) + nack(22) + ack_frame(1, 20, multiple=True)
    return [{1: s}, {2: mixed}, {}, {2: rev}, {}, {2: ack_frame(1, 0)}, {}]


def sc_deliver_cap_bytes(dp):
    """A backlog of large then small bodies drained by an auto-ack and a manual-ack consumer
    under a per-step byte cap: each consumer takes max(1, cap / size of its first delivery)
    a step (StepIn.dcap_bytes), so the drain spreads over steps with ~cap bytes each."""
    dp.set_deliver_cap_bytes(2500)
    dp.declare_queue(VH, "big")
    dp.open_connection(1, VH)
    dp.open_channel(1, 1)
    dp.open_connection(2, VH)
    dp.open_channel(2, 1)
    dp.open_connection(3, VH)
    dp.open_channel(3, 1)
    dp.consume(2, 1, VH, "big", "auto", no_ack=True)
    dp.consume(3, 1, VH, "big", "man", no_ack=False)
    s = publish_stream(14, "", lambda i: "big", 900, seed=11) + publish_stream(30, "", lambda i: "big", 40, seed=12)
    return [{1: s}, {}, {3: ack_frame(1, 0, multiple=True)}, {}, {3: ack_frame(1, 0, multiple=True)}, {}, {}, {}]


SCENARIOS = {
    "deliver_cap_bytes": sc_deliver_cap_bytes,
    "mixed_multiple_settles": sc_mixed_multiple_settles,
    "ring_growth": sc_ring_growth,
    "confirm_ring_full": sc_confirm_ring_full,
    "big_segment": sc_big_segment,
    "window_wrap": sc_window_wrap,
    "tx_hold": sc_tx_hold,
    "basic_get": sc_basic_get,
    "wire_get": sc_wire_get,
    "direct_split": sc_direct_split,
    "default_exchange": sc_default_exchange,
    "topic": sc_topic,
    "fanout": sc_fanout,
    "manual_ack": sc_manual_ack,
    "confirm_mandatory": sc_confirm_mandatory,
    "control_barrier": sc_control_barrier,
    "nack_requeue": sc_nack_requeue,
    "ttl": sc_ttl,
    "frame_error": sc_frame_error,
}

NOW = 1_800_000_000_000


def run(dp, steps, now_step_ms=None):
    """Drive dp through the steps; returns list of normalised per-step outputs."""
    outs = []
    for k, inp in enumerate(steps):
        inp = dict(inp)
        for c in inp.pop("__unpause__", []):
            dp.unpause(c)
        for conn, ch, qn, tag in inp.pop("__consume__", []):   # a consumer attaches between steps
            dp.open_connection(conn, VH)
            dp.open_channel(conn, ch)
            dp.consume(conn, ch, VH, qn, tag, no_ack=True)
        now = NOW + (now_step_ms or 0) * k
        gets = []
        for conn, ch, qn, no_ack in inp.pop("__get__", []):   # Basic.Get between steps
            gets.append(dp.basic_get(conn, ch, dp.queues[(VH, qn)].slot, no_ack, now_ms=now))
        r = dp.step(inp, now_ms=now)
        if isinstance(r, dict):
            eg, ctrl, ev, segs, tx = r["egress"], r["ctrl"], r["events"], r["segs"], r.get("txbuf", [])
        else:
            eg, ctrl, ev, segs, tx = r.egress, r.ctrl, r.events, [s[:4] for s in r.segs], r.txbuf
        outs.append(dict(egress=eg, ctrl=sorted(ctrl), events=sorted(ev),
                         segs=sorted((s[0], s[1], s[2], s[3]) for s in segs), gets=gets, txbuf=sorted(tx)))
    return outs
