"""Scenarios for the sharded data plane.  Each returns a spec that can be applied to
one plane holding every connection (world 1) or to a cluster of ranks (each connection
on one rank, queues placed explicitly).  The single-plane run is the oracle: per-
connection egress must be byte-identical in both layouts (tests/test_sharded*.py)."""

from chanamq_amd.engine.traffic import ack_frame, publish_command, publish_stream

VH = "AMQ.DEFAULT"


class Spec:
    def __init__(self):
        self.exchanges = []      # (name, type)
        self.queues = []         # (name, owner rank, capacity)
        self.binds = []          # (queue, exchange, key)
        self.conns = []          # (rank, conn, [channels])
        self.confirms = []       # (conn, ch)
        self.qos = []            # (conn, ch, prefetch)
        self.consumers = []      # (conn, ch, queue, tag, no_ack)
        self.steps = []          # [{conn: bytes}]
        self.rank_of = {}

    def conn(self, rank, conn, *chs):
        self.conns.append((rank, conn, list(chs)))
        self.rank_of[conn] = rank


def apply(dp, spec, rank=None, world=1, conn_map=None):
    """Configure ``dp`` (rank ``rank`` of ``world``; rank None = the single oracle plane,
    with connection ids renamed through ``conn_map``)."""
    m = conn_map or {}
    if world > 1:
        for name, owner, _ in spec.queues:
            dp.shard_map.place(VH, name, owner % world)
    for name, t in spec.exchanges:
        dp.declare_exchange(VH, name, t)
    for name, _, cap in spec.queues:
        dp.declare_queue(VH, name, capacity=cap)
    for q, x, k in spec.binds:
        dp.bind(VH, q, x, k)
    mine = {c for r, c, _ in spec.conns if rank is None or r % world == rank}
    for r, c, chs in spec.conns:
        if c in mine:
            dp.open_connection(m.get(c, c), VH)
            for ch in chs:
                dp.open_channel(m.get(c, c), ch)
    for c, ch in spec.confirms:
        if c in mine:
            dp.confirm_select(m.get(c, c), ch)
    for c, ch, pf in spec.qos:
        if c in mine:
            dp.qos(m.get(c, c), ch, prefetch_count=pf)
    for c, ch, q, tag, no_ack in spec.consumers:
        if c in mine:
            dp.consume(m.get(c, c), ch, VH, q, tag, no_ack=no_ack)


def split_inputs(spec, step, world):
    out = [dict() for _ in range(world)]
    for c, data in step.items():
        out[spec.rank_of[c] % world][c] = data
    return out


def sp_topic():
    s = Spec()
    s.exchanges.append(("tx", "topic"))
    pats = {"qa": ["forex.*", "*.usd"], "qb": ["*.eur", "forex.*"], "qc": ["*"], "qd": ["quote.#"],
            "qe": ["#"], "qf": ["a.*.c.#.z"]}
    for i, (q, ps) in enumerate(pats.items()):
        s.queues.append((q, i % 3, 1 << 12))
        for p in ps:
            s.binds.append((q, "tx", p))
        s.conn(i % 3, 10 + i, 1)
        s.consumers.append((10 + i, 1, q, "t-" + q, True))
    keys = ["forex.eur", "forex", "trade.jpy", "forex.jpy", "quote", "quote.a.b", "x.usd", "a.b.c.z",
            "a.b.c.q.r.z", "", "forex.", "a..b"]
    for p in range(3):
        s.conn(p, 1 + p, 7)
    s.steps = [{1 + p: publish_stream(24, "tx", lambda i, p=p: keys[(i + p) % len(keys)], 64 + 32 * p,
                                      channel=7, seed=40 + p) for p in range(3)}, {}]
    return s


def sp_fanout_confirm():
    """BASELINE config 3 shape: fanout to many queues spread over the ranks."""
    s = Spec()
    s.exchanges.append(("fx", "fanout"))
    for i in range(8):
        s.queues.append((f"f{i}", i, 1 << 12))
        s.binds.append((f"f{i}", "fx", ""))
        s.conn(i, 20 + i, 1)
        s.consumers.append((20 + i, 1, f"f{i}", f"fc{i}", True))
    s.conn(0, 1, 1)
    s.conn(1, 2, 3)
    s.confirms += [(1, 1), (2, 3)]
    a = publish_stream(12, "fx", lambda i: "k", 700, seed=5)
    b = publish_stream(9, "fx", lambda i: "k", 3000, channel=3, seed=6, frame_max=1024)
    s.steps = [{1: a[:2000], 2: b}, {1: a[2000:]}, {}]
    return s


def sp_direct_manual_ack():
    s = Spec()
    s.exchanges.append(("dx", "direct"))
    for i in range(4):
        s.queues.append((f"w{i}", i, 1 << 12))
        s.binds.append((f"w{i}", "dx", f"k{i}"))
    s.conn(1, 30, 1)
    s.qos.append((30, 1, 6))
    s.consumers += [(30, 1, "w1", "m1", False)]
    s.conn(0, 31, 2)
    s.consumers += [(31, 2, "w0", "m0a", False), (31, 2, "w0", "m0b", False)]
    s.conn(2, 32, 1)
    s.qos.append((32, 1, 3))
    s.consumers += [(32, 1, "w2", "m2", False)]
    s.conn(0, 1, 1)
    s.conn(1, 2, 1)
    p1 = publish_stream(20, "dx", lambda i: f"k{i % 4}", 100, seed=7)
    p2 = publish_stream(20, "dx", lambda i: f"k{(i + 1) % 3}", 50, seed=8)
    s.steps = [{1: p1, 2: p2}, {30: ack_frame(1, 3), 31: ack_frame(2, 4), 32: ack_frame(1, 2)},
               {30: ack_frame(1, 0), 32: ack_frame(1, 0)}, {}]
    return s


def sp_returns():
    """mandatory unroutable (312) and immediate with remote owners (never 313 remotely)."""
    s = Spec()
    s.exchanges.append(("rx", "direct"))
    s.queues += [("r0", 0, 1 << 10), ("r1", 1, 1 << 10)]
    s.binds += [("r0", "rx", "a"), ("r1", "rx", "b")]
    s.conn(1, 40, 1)
    s.consumers.append((40, 1, "r1", "rc", True))
    s.conn(0, 1, 1)
    cmds = []
    for i in range(6):
        key = ["a", "b", "zz"][i % 3]
        cmds.append(publish_command(1, "rx", key, bytes([i]) * 33, {"delivery_mode": 1}, mandatory=True))
    s.steps = [{1: b"".join(cmds)}, {}]
    return s


SHARDED = {"topic": sp_topic, "fanout_confirm": sp_fanout_confirm, "direct_manual_ack": sp_direct_manual_ack,
           "returns": sp_returns}
