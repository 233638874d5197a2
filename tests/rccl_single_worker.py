"""One-rank RCCL run (tests/test_gpu_sharded.py::test_rccl_single_rank_paths): the bench's
exchange code (parallel/exchange.py, device tensors, no host staging) and the engine's
librccl binding (dlopen + every symbol it uses + ncclGetUniqueId) on a real MI355X.  Two
ranks cannot share one device under RCCL, so this is the part of the multi-GPU path a
one-GPU box can execute."""

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    from chanamq_amd.engine.layout import RDESC
    from chanamq_amd.parallel.exchange import Exchanger

    ex = Exchanger()
    assert ex.device_ok and not ex.stage_cpu
    rec = RDESC.itemsize
    g = torch.Generator(device="cuda").manual_seed(5)
    for n_rec, n_pay in ((7, 5000), (0, 0), (300, 333333)):
        sd = torch.randint(0, 256, (max(1, n_rec * rec),), dtype=torch.uint8, device="cuda", generator=g)
        sp = torch.randint(0, 256, (max(1, n_pay),), dtype=torch.uint8, device="cuda", generator=g)
        rd = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
        rp = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
        got = ex.exchange([n_rec, n_pay], sd, sp, rd, rp)
        torch.cuda.synchronize()
        assert got == [n_rec, n_pay], got
        assert torch.equal(rd[:n_rec * rec], sd[:n_rec * rec]) and torch.equal(rp[:n_pay], sp[:n_pay])
    t = torch.arange(8, dtype=torch.float32, device="cuda")
    dist.all_reduce(t)
    torch.cuda.synchronize()
    assert float(t.sum()) == 28.0
    # the engine's own RCCL backend (csrc/kernels/xchg_rccl.h): dlopen librccl, resolve
    # every entry point the sharded server's exchange uses, draw a communicator id
    from chanamq_amd import ops
    uid = ops.load().Engine.xchg_unique_id()
    assert len(uid) == 128
    native = native_lockstep(uid)
    print("RCCL ok: exchanges", ex.calls, "bytes", ex.bytes_sent, "native", native, flush=True)
    dist.destroy_process_group()


def native_lockstep(uid):
    """bench.py's sharded step on the engine-native exchange (``--xchg native``): a world-2
    plane whose live group is this rank alone, so RcclXchg runs on a one-rank communicator
    (CommInitRank, grouped calls, bounded event waits) and the counts go through host shared
    memory, driven by GpuDataPlane.submit_lockstep exactly as the bench drives it.  Rank 1
    is not a member, so its records are dropped; rank 0's queues get their messages."""
    import bench
    from chanamq_amd.engine.dataplane import GpuDataPlane

    cfg = dict(c_max=96, chpc=4, q_max=64, cons_max=256, seg_max=96, cmd_max=1 << 14, deliv_max=1 << 14,
               msg_max=1 << 16, ucap=1024, deliver_cap=4096, ingress_cap=8 << 20, egress_cap=16 << 20,
               log_bytes=256 << 20, ring_pool=1 << 23, tb_max=64, carry_cap=64 << 10)
    dp = GpuDataPlane(device=0, worker=0, world=2, rank=0, native_xchg=1, **cfg)
    dp.xchg_setup("rccl", uid, [0], 10000, counts_shm=f"cmq-rccl-test-{os.getpid()}")
    pool, segs, offs, blens, mps, _, _ = bench.build_workload(dp, 0, 64, 4, 1024, 8192, 4, cons_base=64,
                                                              shards=2)
    base = pool.ctypes.data
    delivered = published = 0
    pending = []
    for i in range(12):
        b = i % len(segs)
        pending.append(dp.submit_lockstep(segs[b], base + offs[b], blens[b]))
        if len(pending) > 1:
            c = dp.finish(pending.pop(0), collect=False).counters
            delivered += c["n_deliv"]
            published += c["n_pubs"]
    for t in pending:
        c = dp.finish(t, collect=False).counters
        delivered += c["n_deliv"]
        published += c["n_pubs"]
    dp.eng.sync()
    # about half the publishes route to rank 0's 4 queues (the rest to rank 1: dropped)
    assert published == 12 * round(mps) and 0.3 * published < delivered < 0.7 * published, (published, delivered)
    ht = dp.eng.host_times(False)
    return {"published": published, "delivered": delivered, "exchange_us_per_step": round(ht["exchange"] * 1e6 / 12, 1)}


if __name__ == "__main__":
    main()
