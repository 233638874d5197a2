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

from ..engine.layout import RDESC

REC = RDESC.itemsize
_RT = []


def _roctx():
    """The data-plane extension's roctx hooks when it is already loaded (GPU runs), else None."""
    if not _RT:
        import sys
        _RT.append(sys.modules.get("chanamq_amd.ops._dataplane"))
    return _RT[0]


class Exchanger:
    def __init__(self, comm=None, stage_cpu=None):
        from .comm import Comm
        self.comm = comm or Comm()
        self.device_ok = self.comm.backend == "nccl"
        self.stage_cpu = (not self.device_ok) if stage_cpu is None else stage_cpu
        self.bytes_sent = 0
        self.calls = 0

    @property
    def world(self):
        return self.comm.world

    @property
    def rank(self):
        return self.comm.rank

    def _a2a(self, out, inp, out_splits, in_splits):
        if self.stage_cpu and inp.is_cuda:
            ci, co = inp.cpu(), torch.empty(out.numel(), dtype=out.dtype)
            self.comm.alltoall(co, ci, out_splits, in_splits)
            out.copy_(co)
        else:
            self.comm.alltoall(out, inp, out_splits, in_splits)

    def exchange(self, send_counts, send_desc, send_pay, recv_desc, recv_pay):
        """``send_counts`` = [n_0..n_{W-1}, b_0..b_{W-1}] (logical ranks) -> received
        [n.., b..] by source.  Tensors are flat uint8 (records: 64 bytes each).  Traffic
        for ranks that left the group is dropped (its owner is gone; at-most-once)."""
        rt = _roctx()
        if rt is not None:
            rt.roctx_push("chanamq.X1.all_to_all")
        try:
            return self._exchange(send_counts, send_desc, send_pay, recv_desc, recv_pay)
        finally:
            if rt is not None:
                rt.roctx_pop()

    def _exchange(self, send_counts, send_desc, send_pay, recv_desc, recv_pay):
        W = self.world
        live = set(self.comm.members)
        n = [send_counts[r] if r in live else 0 for r in range(W)]
        b = [send_counts[W + r] if r in live else 0 for r in range(W)]
        if n != list(send_counts[:W]):
            # repack without the departed destinations (records are destination-major)
            n, b, send_desc, send_pay = _drop_dead(send_counts, send_desc, send_pay, live, W)
        rc = self.comm.alltoall_counts([[n[r], b[r]] for r in range(W)])
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


def _drop_dead(send_counts, send_desc, send_pay, live, W):
    n0, b0 = list(send_counts[:W]), list(send_counts[W:2 * W])
    descs, pays, n, b = [], [], [], []
    do = po = 0
    for r in range(W):
        if r in live:
            descs.append(send_desc[do:do + n0[r] * REC])
            pays.append(send_pay[po:po + b0[r]])
            n.append(n0[r])
            b.append(b0[r])
        else:
            n.append(0)
            b.append(0)
        do += n0[r] * REC
        po += b0[r]
    return n, b, torch.cat(descs) if descs else send_desc[:0], torch.cat(pays) if pays else send_pay[:0]


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
