#!/usr/bin/env python3
"""Per-GPU kernel work of the sharded headline step at world size W, measured on ONE GPU.

The driver's multi-GPU bench (bench.py under torch.distributed.run, one rank per MI355X,
RCCL all-to-all) cannot run here: RCCL refuses two ranks on one device.  This script
builds the same W ranks as in-process planes on one device (parallel/cluster.py style:
the all-to-all becomes device copies), runs bench.py's config-2 workload for each rank,
and steps them one after another, so under ``rocprofv3 --kernel-trace --stats`` every
kernel of every rank is timed without another rank's kernels competing for the CUs.

    rocprofv3 --kernel-trace --stats -d out -- python3 bench/world_rehearsal.py --world 8

Kernel time per rank-step = (sum of the data-plane kernels) / (steps x world): the compute
one GPU of a W-GPU node spends per step, to set against the step's PCIe time (16.7 MB each
way, ~380 us at the measured ~44 GB/s per direction).  Prints one JSON line (host wall
time per rank-step included, which is NOT a throughput: the ranks share one GPU).
"""

import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--producers", type=int, default=256)
    ap.add_argument("--queues", type=int, default=16)
    ap.add_argument("--chunk", type=int, default=65536)
    ap.add_argument("--blocks", type=int, default=8)
    ap.add_argument("--log-gib", type=int, default=2)
    args = ap.parse_args()

    import bench
    from chanamq_amd.engine.dataplane import GpuDataPlane
    from chanamq_amd.parallel.exchange import local_exchange
    from chanamq_amd.parallel.shard import ShardMap

    W, P, Q = args.world, args.producers, args.queues
    qtot = Q * W
    sm = ShardMap(W)
    cfg = dict(c_max=max(1024, P + Q + 1), chpc=4, q_max=max(64, qtot + 64), cons_max=max(1024, Q + 16),
               seg_max=max(1024, P + Q), cmd_max=1 << 17, deliv_max=1 << 16, msg_max=1 << 22, ucap=4096,
               deliver_cap=8192, ingress_cap=max(32 << 20, P * args.chunk + (4 << 20)), egress_cap=128 << 20,
               log_bytes=args.log_gib << 30, ring_pool=Q * (1 << 20) + qtot + 1024, tb_max=max(64, qtot),
               fan_max=max(1 << 20, qtot * 2), carry_cap=256 << 10)
    planes, work = [], []
    for r in range(W):
        dp = GpuDataPlane(device=0, worker=r, world=W, rank=r, shard_map=sm, exchange_lag=1, **cfg)
        planes.append(dp)
        work.append(bench.build_workload(dp, r, P, Q, 1024, args.chunk, args.blocks, cons_base=P, shards=W))

    step_i = 0
    delivered = 0

    def step():
        nonlocal step_i, delivered
        b = step_i % args.blocks
        tickets = []
        for r, dp in enumerate(planes):
            pool, segs, offs, blens = work[r][:4]
            tickets.append(dp.submit_raw(segs[b], pool.ctypes.data + offs[b], blens[b]))
        recv = local_exchange(planes) if W > 1 else None   # world 1: no phase B
        for r, dp in enumerate(planes):
            if recv is not None:
                dp.set_import(recv[r])
            res = dp.finish(tickets[r], collect=False, wait_egress=True)
            delivered += res.counters["n_deliv"]
        step_i += 1

    for _ in range(args.warmup):
        step()
    delivered = 0
    import torch
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    cross = sum(p.exchanger.bytes_sent if p.exchanger else 0 for p in planes)
    print(json.dumps({"world": W, "steps": args.steps, "rank_steps": args.steps * W,
                      "deliveries_per_rank_step": delivered / (args.steps * W),
                      "host_ms_per_rank_step_shared_gpu": 1000 * t / (args.steps * W),
                      "note": "W ranks stepped one after another on one GPU; kernel time per rank-step "
                              "comes from rocprofv3 kernel stats / (steps x world)", "cross_bytes": cross}))


if __name__ == "__main__":
    main()
