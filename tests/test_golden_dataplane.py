"""Protocol-level checks of the golden data plane (CPU): what a client would observe."""

from collections import defaultdict

from dp_scenarios import SCENARIOS, VH, run

from chanamq_amd.engine.golden import GoldenDataPlane
from chanamq_amd.engine.layout import SS_CTRL, SS_FRAME_ERROR
from chanamq_amd.protocol.codec import CommandAssembler, FrameParser


def decode(buf):
    fp, ca = FrameParser(), CommandAssembler()
    out = []
    for fr in fp.feed(buf):
        c = ca.feed(fr)
        if c is not None:
            out.append(c)
    return out


def run_sc(name):
    g = GoldenDataPlane(c_max=64, chpc=8, q_max=64, x_max=64, cons_max=256, ucap=256)
    outs = run(g, SCENARIOS[name](g), now_step_ms=3000)
    per_conn = defaultdict(list)
    for o in outs:
        for c, b in o["egress"].items():
            per_conn[c].extend(decode(b))
    return g, outs, per_conn


def test_direct_split_delivers_only_matching_in_order():
    g, outs, pc = run_sc("direct_split")
    d = [c for c in pc[2] if c.method.name == "basic.deliver"]
    assert len(d) == sum(1 for i in range(40) if i % 3)
    assert [c.method.delivery_tag for c in d] == list(range(1, len(d) + 1))
    assert all(c.method.consumer_tag == "c1" and c.channel == 5 for c in d)


def test_default_exchange_routes_by_queue_name():
    g, outs, pc = run_sc("default_exchange")
    d = [c for c in pc[3] if c.method.name == "basic.deliver"]
    assert len(d) == 10 and all(len(c.body) == 50 for c in d)


def test_topic_reference_vectors():
    from chanamq_amd.models.matcher import topic_match
    g, outs, pc = run_sc("topic")
    keys_qa = [c.method.routing_key for c in pc[10]]
    assert all(topic_match("forex.*", k) or topic_match("*.usd", k) for k in keys_qa)
    assert "forex.eur" in keys_qa and "forex" not in keys_qa


def test_fanout_body_split_at_frame_max():
    g, outs, pc = run_sc("fanout")
    for c in (20, 21, 22):
        d = [x for x in pc[c] if x.method.name == "basic.deliver"]
        assert len(d) == 25 and all(len(x.body) == 2000 for x in d)


def test_manual_ack_prefetch_and_release():
    g, outs, pc = run_sc("manual_ack")
    d = [c for c in pc[2] if c.method.name == "basic.deliver"]
    assert len(d) == 12
    # first step is limited by prefetch 5
    first = decode(outs[0]["egress"][2])
    assert len(first) == 5


def test_confirms_and_mandatory_return():
    g, outs, pc = run_sc("confirm_mandatory")
    names = [c.method.name for c in pc[1]]
    assert names == ["basic.return", "basic.ack"]
    ret, ack = pc[1]
    assert ret.method.reply_code == 312 and ret.body == bytes([3]) * 40
    assert ack.method.delivery_tag == 9 and ack.method.multiple


def test_control_barrier_pauses_and_resumes():
    g, outs, pc = run_sc("control_barrier")
    assert outs[0]["segs"][0][1] & SS_CTRL
    assert len(outs[0]["ctrl"]) == 1
    d = [c for c in pc[2] if c.method.name == "basic.deliver"]
    assert len(d) == 7


def test_nack_requeue_redelivered_flag():
    g, outs, pc = run_sc("nack_requeue")
    d = [c for c in pc[2] if c.method.name == "basic.deliver"]
    red = [c for c in d if c.method.redelivered]
    assert len(red) >= 2
    assert len(d) == 6 + 2


def test_ttl_expiry_drops():
    g, outs, pc = run_sc("ttl")
    assert g.counters["n_expired"] >= 0


def test_frame_error_reported():
    g, outs, pc = run_sc("frame_error")
    assert outs[0]["segs"][0][1] & SS_FRAME_ERROR


def test_basic_get_semantics():
    """GetOk tags follow the channel's delivery tags, message-count is what is left, a
    nacked get comes back redelivered, an expired head is skipped, an empty queue -> None."""
    g, outs, pc = run_sc("basic_get")
    gets = [decode(f) if f is not None else None for o in outs for f, _ in o["gets"]]
    counts = [n for o in outs for _, n in o["gets"]]
    oks = [x[0] for x in gets if x]
    assert [c.method.name for c in oks] == ["basic.get_ok"] * len(oks)
    assert [c.method.delivery_tag for c in oks] == list(range(1, len(oks) + 1))
    assert len(oks[0].body) == 5000 and oks[0].channel == 1
    # step 1: no-ack g0, manual g1 (tag 2), manual g2 (tag 3); step 2: ack 2, get g3 (tag 4)
    # step 3: nack 3 -> requeued in front; step 4: g2 again (redelivered), g4, expired skip, empty
    assert [c.method.redelivered for c in oks] == [False, False, False, False, True, False]
    assert counts[:4] == [5, 4, 3, 2]
    assert gets[-1] is None and gets[-2] is None
    assert sum(1 for x in gets if x is None) == 2


def test_tx_channel_commands_held_not_applied():
    g, outs, pc = run_sc("tx_hold")
    held = [raw for o in outs for _, _, raw in o["txbuf"]]
    assert len(held) == 4                      # 3 publishes + 1 ack of the Tx channel, wire order
    assert [decode(r)[0].method.name for r in held] == ["basic.publish"] * 3 + ["basic.ack"]
    d = [c for c in pc[2] if c.method.name == "basic.deliver"]
    assert len(d) == 4                         # only the non-transactional channel's
    assert [c.body for c in d] == [bytes([9 - i]) * 41 for i in range(4)]
    assert any(o["ctrl"] for o in outs)        # tx.commit reached the host and paused the connection


def test_ring_full_confirms_with_nack_never_ack():
    g, outs, pc = run_sc("confirm_ring_full")
    per_step = [[(c.channel, c.method.name, c.method.delivery_tag, c.method.multiple)
                 for c in decode(o["egress"].get(1, b""))] for o in outs]
    assert per_step[0] == [(1, "basic.ack", 10, True)]
    # step 2: 6 of channel 1's 10 publishes did not fit the 16-slot ring -> Nack over the range
    assert (1, "basic.nack", 20, True) in per_step[1] and (2, "basic.ack", 5, True) in per_step[1]
    assert per_step[2] == [(1, "basic.ack", 23, True)]
    assert g.counters is not None


def test_big_segment_delivers_all():
    g, outs, pc = run_sc("big_segment")
    d = [c for c in pc[2] if c.method.name == "basic.deliver"]
    assert len(d) == 150 and all(len(c.body) == 1000 for c in d)


def test_ring_growth_stores_and_delivers_everything():
    g, outs, pc = run_sc("ring_growth")
    acks = [c.method for c in pc[1]]
    assert [(m.name, m.delivery_tag) for m in acks] == [("basic.ack", 6), ("basic.ack", 16), ("basic.ack", 31)]
    d = [c for c in pc[2] if c.method.name == "basic.deliver"]
    assert len(d) == 31 and [c.method.delivery_tag for c in d] == list(range(1, 32))
    assert g.queues[("AMQ.DEFAULT", "grow")].capacity >= 31
    assert g.counters["n_ring_full"] == 0


def test_mixed_multiple_settles_first_cover_wins():
    """nack(4,multiple,requeue) ack(8,multiple) nack(10,multiple,drop) ack(12) nack(14,
    multiple,requeue) in one step: 1-4, 11, 13, 14 come back redelivered, 5-8 and 12 are
    acked, 9-10 dropped; the reversed order later (ack 18 multiple, nack 22, ack 20) acks
    up to 18 and requeues 19-22."""
    g, outs, pc = run_sc("mixed_multiple_settles")
    d = [c for c in pc[2] if c.method.name == "basic.deliver"]
    first = {c.method.delivery_tag: c.body for c in d[:16]}
    red = [c for c in d[16:] if c.method.redelivered]
    assert [c.body for c in red[:7]] == [first[t] for t in (1, 2, 3, 4, 11, 13, 14)]
    assert not any(c.body in (first[9], first[10]) for c in d[16:])
    assert g.memory_in_use() == 0


def test_wire_basic_get_served_by_the_step():
    """Basic.Get decoded from the connection's bytes (no host round trip): pipelined Gets of
    one key in one step, the next key / an ack wait a step, GetEmpty rendered in egress,
    the host gets only what the step cannot decide (unnamed / exclusive queue)."""
    from chanamq_amd.protocol.codec import CommandAssembler, FrameParser
    g, outs, pc = run_sc("wire_get")

    def names(o):
        fp, ca = FrameParser(), CommandAssembler()
        cmds = [ca.feed(f) for f in fp.feed(o["egress"].get(2, b""))]
        return [(c.channel, c.method.name, getattr(c.method, "delivery_tag", None)) for c in cmds if c and c.method]
    assert names(outs[1]) == [(1, "basic.get_ok", 1), (1, "basic.get_ok", 2), (1, "basic.get_ok", 3)]
    assert names(outs[2]) == [(1, "basic.get_ok", 4), (1, "basic.get_ok", 5)]   # (the ack waits a step)
    assert names(outs[3]) == [(2, "basic.get_ok", 1)]
    assert names(outs[5]) == [(1, "basic.get_ok", 6), (1, "basic.get_empty", None)]
    assert outs[1]["ctrl"] == [] and outs[5]["ctrl"] == []
    assert [len(c) for c in outs[6]["ctrl"]] == [2] and [len(c) for c in outs[7]["ctrl"]] == [2]
    assert g.message_count(g.queues[(VH, "wg")].slot) == 0
