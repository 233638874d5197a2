"""One rank of the engine-native exchange test (tests/test_gpu_sharded.py): a sharded plane
built with native_xchg=1 driven the way the sharded server's stepper drives it
(GpuDataPlane.submit_lockstep: phase A, the previous step's exchange, phase B) over the
engine's RCCL backend (RcclXchg through CHANAMQ_RCCL_LIB = the tests' stand-in: RCCL
refuses several ranks on one GPU) or its shared-memory backend.  argv: scenario out_dir
rccl|shm [counts_shm].  Writes rank<r>.json: per step {conn: egress hex}."""

import json
import os
import sys
import uuid

import torch.distributed as dist

from sharded_scenarios import SHARDED, apply, split_inputs


def main():
    name, out, kind = sys.argv[1], sys.argv[2], sys.argv[3]
    counts_shm = len(sys.argv) > 4 and sys.argv[4] == "counts_shm"
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    import torch
    torch.cuda.set_device(0)
    from chanamq_amd.engine.dataplane import GpuDataPlane
    from gpu_cfg import CFG
    dp = GpuDataPlane(world=world, rank=rank, native_xchg=1, **CFG)
    names = [None]
    if rank == 0:
        tag = f"cmq-nx-{os.getpid()}-{uuid.uuid4().hex[:8]}"
        names = [{"uid": dp.xchg_unique_id() if kind == "rccl" else None, "shm": tag}]
    dist.broadcast_object_list(names, src=0)
    nm = names[0]
    if kind == "rccl":
        dp.xchg_setup("rccl", nm["uid"], list(range(world)), 20000, counts_shm=nm["shm"] + "-c" if counts_shm else "")
        assert dp.eng.info()["rccl_standin"] == 1, "expected the tests' RCCL stand-in"
    else:
        dp.xchg_setup("shm", nm["shm"], list(range(world)), 20000)
    spec = SHARDED[name]()
    apply(dp, spec, rank=rank, world=world)
    res = []
    for k, st in enumerate(spec.steps + [{}] * 2):
        segs, ptr, n = dp.stage(split_inputs(spec, st, world)[rank])
        t = dp.submit_lockstep(segs, ptr, n, now_ms=1000 + k)
        r = dp.finish(t, collect=True)
        res.append({str(c): b.hex() for c, b in r.egress.items()})
    with open(os.path.join(out, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
