"""Cross-rank publish exchange: one all-to-all per step over RCCL (xGMI) or gloo.

Each step of a sharded data plane produces, per destination rank r, ``n_r`` 64-byte
records (``RDesc``) and ``b_r`` payload bytes, packed destination-major on the device
(dataplane.hip k_pack).  ``Exchanger.exchange`` moves them with three collectives:

1. ``all_to_all_single`` of the (n_r, b_r) count pairs (int64, equal splits);
2. ``all_to_all_single`` of the record bytes with per-rank splits;
3. ``all_to_all_single`` of the payload bytes with per-rank splits.

With the NCCL backend (= RCCL on ROCm) the operands are device tensors and the copies
run over xGMI without touching the host; with gloo they are CPU tensors (the CPU test
path), or device tensors staged through the host (``stage_cpu``: multi-process tests
that share one GPU, where RCCL refuses two ranks on one device).

The reference moves messages between nodes with Akka remoting per message
(chana-mq-server/.../engine/QueueEntity.scala push/pull over cluster sharding); here a
step's whole cross-rank traffic is one bulk collective.
"""

import torch
import torch.distributed as dist

from ..engine.layout import RDESC

REC = RDESC.itemsize


class Exchanger:
    def __init__(self, world=None, rank=None, group=None, stage_cpu=None):
        self.group = group
        self.world = dist.get_world_size(group) if world is None else world
        self.rank = dist.get_rank(group) if rank is None else rank
        backend = dist.get_backend(group)
        self.device_ok = backend == "nccl"
        self.stage_cpu = (not self.device_ok) if stage_cpu is None else stage_cpu
        self.bytes_sent = 0
        self.calls = 0

    def _a2a(self, out, inp, out_splits, in_splits):
        if self.stage_cpu and inp.is_cuda:
            ci, co = inp.cpu(), torch.empty(out.numel(), dtype=out.dtype)
            dist.all_to_all_single(co, ci, out_splits, in_splits, group=self.group)
            out.copy_(co)
        else:
            dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)

    def exchange(self, send_counts, send_desc, send_pay, recv_desc, recv_pay):
        """``send_counts`` = [n_0..n_{W-1}, b_0..b_{W-1}] -> received [n.., b..] by source.
        Tensors are flat uint8 (records: 64 bytes each)."""
        W = self.world
        n, b = list(send_counts[:W]), list(send_counts[W:2 * W])
        dev = send_desc.device if (self.device_ok and send_desc.is_cuda) else torch.device("cpu")
        cnt = torch.tensor([v for r in range(W) for v in (n[r], b[r])], dtype=torch.int64, device=dev)
        out = torch.empty_like(cnt)
        dist.all_to_all_single(out, cnt, group=self.group)
        rc = out.view(W, 2).cpu().tolist()
        rn, rb = [x[0] for x in rc], [x[1] for x in rc]
        if sum(rn) * REC > recv_desc.numel() or sum(rb) > recv_pay.numel():
            raise RuntimeError(f"rank {self.rank}: received {sum(rn)} records / {sum(rb)} bytes "
                               "exceed the import buffers")
        sd, rd = sum(n) * REC, sum(rn) * REC
        self._a2a(recv_desc[:rd], send_desc[:sd], [x * REC for x in rn], [x * REC for x in n])
        self._a2a(recv_pay[:sum(rb)], send_pay[:sum(b)], rb, b)
        self.bytes_sent += sd + sum(b)
        self.calls += 1
        return rn + rb


def local_exchange(planes):
    """In-process all-to-all between the planes of a ``LocalCluster`` (one device or
    CPU): rank r's region for destination s is copied into s's receive buffers in
    source order — the exact layout ``Exchanger.exchange`` produces."""
    W = len(planes)
    sends = [p.pending_send_counts() for p in planes]
    recv = []
    for s in range(W):
        rn = [sends[r][s] for r in range(W)]
        rb = [sends[r][W + s] for r in range(W)]
        dd = planes[s].xfer_recv_desc()
        dp = planes[s].xfer_recv_pay()
        od = op = 0
        for r in range(W):
            n, b = sends[r][:W], sends[r][W:2 * W]
            d0 = sum(n[:s]) * REC
            p0 = sum(b[:s])
            sd, sp = planes[r].xfer_send_desc(), planes[r].xfer_send_pay()
            if rn[r]:
                dd[od:od + rn[r] * REC] = sd[d0:d0 + rn[r] * REC]
            if rb[r]:
                dp[op:op + rb[r]] = sp[p0:p0 + rb[r]]
            od += rn[r] * REC
            op += rb[r]
        recv.append(rn + rb)
    return recv
