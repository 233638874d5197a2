"""One rank of the multi-process sharded-node tests (gloo, golden planes).
argv: scenario out_dir [die_rank die_after_step]"""

import json
import os
import struct
import sys

import torch.distributed as dist

from chanamq_amd.engine.golden import GoldenDataPlane
from chanamq_amd.engine.traffic import publish_stream
from chanamq_amd.parallel.comm import Comm
from chanamq_amd.parallel.node import ShardedNode

VH = "AMQ.DEFAULT"


def count_delivers(b):
    n = pos = 0
    while pos + 7 <= len(b):
        t, _, size = struct.unpack_from(">BHI", b, pos)
        if t == 1 and b[pos + 7:pos + 11] == b"\x00\x3c\x00\x3c":
            n += 1
        pos += 8 + size
    return n


def durable(out, die_rank, die_after):
    """Persistent messages on durable queues survive their rank: nobody consumes until
    after the failover, then every message published by any rank (including the ones
    only rank ``die_rank``'s store held) is delivered once by the queues' new owners."""
    from chanamq_amd.broker import load
    from chanamq_amd.engine.persistence import GpuPersistence
    core = load()
    rank, world = dist.get_rank(), dist.get_world_size()

    def open_store(r):
        st = core.Store()
        os.makedirs(os.path.join(out, "store"), exist_ok=True)
        st.open(os.path.join(out, "store", f"rank{r}"), False)
        return st

    plane = GoldenDataPlane(default_queue_capacity=1 << 12, ring_pool=1 << 22, world=world, rank=rank, persist=True)
    store = open_store(rank)
    pers = GpuPersistence(plane, store)
    node = ShardedNode(plane, Comm(timeout_s=20), hb_timeout_s=1.0, persistence=pers, peer_store=open_store)
    nq, steps, per_step = 6, 8, 5
    if rank == 0:
        node.submit("declare_exchange", VH, "dfx", "fanout", durable=True)
        for i in range(nq):
            node.submit("declare_queue", VH, f"d{i}", durable=True)
            node.submit("bind", VH, f"d{i}", "dfx", "")
    node.step({}, now_ms=1)
    for q in plane.queues.values():   # every rank records the durable topology (server: declare)
        pers.queue(q)
    store.sync()
    plane.open_connection(1, VH)
    plane.open_channel(1, 1)
    got, cons = {}, {}
    for k in range(steps + 6):
        if rank == die_rank and k == die_after:
            os._exit(0)
        if k >= steps:   # drain: consumers on whatever this rank owns now
            for q in plane.queues.values():
                if q.owner == rank and q.name not in cons:
                    c = 200 + int(q.name[1:])
                    plane.open_connection(c, VH)
                    plane.open_channel(c, 1)
                    plane.consume(c, 1, VH, q.name, "c-" + q.name, no_ack=True)
                    cons[q.name] = c
        data = publish_stream(per_step, "dfx", lambda i: "", 40, persistent=True,
                              seed=rank * 100 + k) if k < steps else b""
        res, _ = node.step({1: data} if data else {}, now_ms=1000 + k)
        pers.after_step()
        pers.commit()
        for c, b in res["egress"].items():
            if c in cons.values():
                got[str(c)] = got.get(str(c), 0) + count_delivers(b)
    owned = sorted(q.name for q in plane.queues.values() if q.owner == rank)
    with open(os.path.join(out, f"rank{rank}.json"), "w") as f:
        json.dump({"owned": owned, "failovers": node.failovers, "live": sorted(node.members.live),
                   "deliveries": got, "rows": store.row_count("queues")}, f)
    node.comm.barrier()   # the c10d store lives in rank 0: nobody leaves while others still use it
    node.close()
    store.close()


def links(out, die_rank, die_after):
    """Remote consumer across a failure.  Queue lq lives on rank 2, its consumer on rank 1
    (a link), the publisher on rank 0 (which also hosts the c10d store, so it must live).
    die_rank 1 (the consumer's rank): the owner closes the link, everything the consumer
      held (it never acks) returns to lq and a new consumer on rank 2 gets every message.
    die_rank 2 (the owner): lq re-homes and the link re-attaches at the new owner; the
      consumer keeps receiving what is published after the failover."""
    rank, world = dist.get_rank(), dist.get_world_size()
    plane = GoldenDataPlane(default_queue_capacity=1 << 12, ring_pool=1 << 22, world=world, rank=rank)
    node = ShardedNode(plane, Comm(timeout_s=20), hb_timeout_s=1.0)
    if rank == 0:
        node.submit("declare_exchange", VH, "lx", "direct")
        node.submit("place_queue", VH, "lq", 2)
        node.submit("declare_queue", VH, "lq")
        node.submit("bind", VH, "lq", "lx", "k")
    node.step({}, now_ms=1)
    if rank == 1:
        node.submit("link_open", 7, VH, "lq", 1, 1000)
    node.step({}, now_ms=2)
    if rank == 1:
        plane.open_connection(20, VH)
        plane.open_channel(20, 1)
        plane.consume(20, 1, VH, node.links.shadow_of(7), "remote", no_ack=(die_rank == 2))
    plane.open_connection(1, VH)
    plane.open_channel(1, 1)
    got, steps, per = {}, 10, 5
    local = False
    for k in range(steps + 4):
        if rank == die_rank and k == die_after:
            os._exit(0)
        if k == steps and die_rank == 1 and rank == 2:   # after the failover: drain lq here
            plane.open_connection(30, VH)
            plane.open_channel(30, 1)
            plane.consume(30, 1, VH, "lq", "local", no_ack=True)
            local = True
        data = publish_stream(per, "lx", lambda i: "k", 40, seed=k) if (rank == 0 and k < steps) else b""
        res, _ = node.step({1: data} if data else {}, now_ms=1000 + k)
        for c, b in res["egress"].items():
            got[str(c)] = got.get(str(c), 0) + count_delivers(b)
    with open(os.path.join(out, f"rank{rank}.json"), "w") as f:
        json.dump({"deliveries": got, "failovers": node.failovers, "links": sorted(node.links.links),
                   "local": local, "live": sorted(node.members.live)}, f)
    node.comm.barrier()
    node.close()


def main():
    scen, out = sys.argv[1], sys.argv[2]
    die_rank = int(sys.argv[3]) if len(sys.argv) > 3 else -1
    die_after = int(sys.argv[4]) if len(sys.argv) > 4 else -1
    dist.init_process_group("gloo")
    if scen == "durable":
        return durable(out, die_rank, die_after)
    if scen == "links":
        return links(out, die_rank, die_after)
    rank, world = dist.get_rank(), dist.get_world_size()
    plane = GoldenDataPlane(default_queue_capacity=1 << 12, ring_pool=1 << 22, world=world, rank=rank)
    node = ShardedNode(plane, Comm(timeout_s=20), hb_timeout_s=1.0)
    nq = 6
    # replicated topology through the control log (issued by rank 0 only)
    if rank == 0:
        node.submit("declare_exchange", VH, "fx", "fanout")
        for i in range(nq):
            node.submit("declare_queue", VH, f"q{i}")
            node.submit("bind", VH, f"q{i}", "fx", "")
    node.step({}, now_ms=1)
    cons = {}

    def attach_consumers():
        for q in plane.queues.values():
            if q.owner == rank and q.name not in cons:
                c = 100 + int(q.name[1:])
                plane.open_connection(c, VH)
                plane.open_channel(c, 1)
                plane.consume(c, 1, VH, q.name, "c-" + q.name, no_ack=True)
                cons[q.name] = c

    attach_consumers()
    plane.open_connection(1, VH)
    plane.open_channel(1, 1)
    got = {}
    steps = 8
    for k in range(steps):
        if rank == die_rank and k == die_after:
            os._exit(0)           # abrupt failure at a step boundary
        data = publish_stream(5, "fx", lambda i: "k", 40, seed=rank * 100 + k)
        res, _ = node.step({1: data}, now_ms=1000 + k)
        for c, b in res["egress"].items():
            got[str(c)] = got.get(str(c), 0) + count_delivers(b)
        attach_consumers()
    owned = sorted(q.name for q in plane.queues.values() if q.owner == rank)
    with open(os.path.join(out, f"rank{rank}.json"), "w") as f:
        json.dump({"owned": owned, "failovers": node.failovers, "live": sorted(node.members.live),
                   "deliveries": got}, f)
    node.comm.barrier()
    node.close()


if __name__ == "__main__":
    main()
    # leave without running C++ destructors: a process group torn down at interpreter exit
    # (while gloo / store threads still run) can abort with std::terminate
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(0)
