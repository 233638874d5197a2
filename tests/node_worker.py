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


def main():
    scen, out = sys.argv[1], sys.argv[2]
    die_rank = int(sys.argv[3]) if len(sys.argv) > 3 else -1
    die_after = int(sys.argv[4]) if len(sys.argv) > 4 else -1
    dist.init_process_group("gloo")
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
    node.close()


if __name__ == "__main__":
    main()
