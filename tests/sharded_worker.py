"""One rank of a multi-process sharded data-plane test (launched by the tests with
RANK/WORLD_SIZE/MASTER_* set).  argv: scenario out_dir golden|gpu [lag]

``lag``: pipelined exchange (exchange_lag=1: each step's all-to-all runs while the next
step's ingress is copied, and is imported by that next step); two empty steps flush it."""

import json
import os
import sys

import torch.distributed as dist

from chanamq_amd.parallel.exchange import Exchanger
from sharded_scenarios import SHARDED, apply, split_inputs


def main():
    name, out, kind = sys.argv[1], sys.argv[2], sys.argv[3]
    lag = len(sys.argv) > 4 and sys.argv[4] == "lag"
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    ex = Exchanger()
    spec = SHARDED[name]()
    if kind == "golden":
        from chanamq_amd.engine.golden import GoldenDataPlane
        dp = GoldenDataPlane(default_queue_capacity=1 << 12, ring_pool=1 << 20, world=world, rank=rank,
                             exchanger=ex)
    else:
        import torch
        torch.cuda.set_device(0)
        from chanamq_amd.engine.dataplane import GpuDataPlane
        from gpu_cfg import CFG
        dp = GpuDataPlane(world=world, rank=rank, exchanger=ex, exchange_lag=int(lag), **CFG)
    apply(dp, spec, rank=rank, world=world)
    res = []
    for k, st in enumerate(spec.steps + [{}] * (2 if lag else 0)):
        r = dp.step(split_inputs(spec, st, world)[rank], now_ms=1000 + k)
        eg = r["egress"] if isinstance(r, dict) else r.egress
        res.append({str(c): b.hex() for c, b in eg.items()})
    with open(os.path.join(out, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
