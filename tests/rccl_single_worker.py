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
    print("RCCL ok: exchanges", ex.calls, "bytes", ex.bytes_sent, flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
