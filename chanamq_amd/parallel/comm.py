"""Collectives between the live ranks of a sharded broker.

``Comm`` wraps a c10d ProcessGroup (RCCL on GPUs, gloo on CPU) and maps *logical* rank
ids (stable for the life of the node; queue ownership and pair ordering use them) to the
members of the current group.  After a membership change (parallel/membership.py) the
survivors build a fresh group over a new store prefix (``rebuild``): no collective on
the old communicator is needed, so a dead peer cannot block the rebuild — the failure
handling the reference gets from Akka Cluster (C41/C42) re-done for collectives.
"""

import datetime
import json

import torch
import torch.distributed as dist


class Comm:
    def __init__(self, pg=None, rank=None, world=None, store=None, backend=None, device=None, timeout_s=60,
                 wait_s=None):
        if pg is None:
            pg = dist.distributed_c10d._get_default_group()
            rank = dist.get_rank() if rank is None else rank
            world = dist.get_world_size() if world is None else world
            store = store or dist.distributed_c10d._get_default_store()
            backend = backend or dist.get_backend()
        self.pg, self.store = pg, store
        self.rank = rank                    # logical id of this process
        self.world = world                  # logical world (fixed)
        self.members = list(range(world))   # live logical ranks, ordered = group ranks
        self.backend = backend or "gloo"
        self.device = device
        self.timeout_s = timeout_s
        # RCCL: Work.wait(timeout) blocks the host and raises when a peer stops answering
        # (without it the wait only orders streams and a dead peer hangs the GPU stream).
        # Opt-in (the failover-capable sharded server sets it; the benchmark keeps the
        # plain stream-ordered waits)
        self.wait_s = wait_s
        self.epoch = 0

    def _wait(self, work, block=True):
        """RCCL: ``block`` = wait on the host with a timeout (a lost peer raises here and
        the node fails over); otherwise only order the current stream behind the
        collective (the bulk payload all-to-all, which must not stall the host: the
        per-step count exchange before it already detects a lost peer)."""
        if self.backend == "nccl" and block and self.wait_s:
            if not work.wait(datetime.timedelta(seconds=self.wait_s)):
                raise RuntimeError("collective timed out (peer lost)")
        else:
            work.wait()

    # ---------------------------------------------------------------- membership
    @property
    def group_rank(self):
        return self.members.index(self.rank)

    def rebuild(self, live):
        """New communicator over the surviving logical ranks ``live`` (every survivor
        calls this with the same set)."""
        live = sorted(live)
        if self.rank not in live:
            raise RuntimeError("this rank is not in the live set")
        self.epoch += 1
        if self.backend == "nccl":   # free the old communicator's stuck kernels / streams
            try:
                self.pg.abort()
            except Exception:   # already torn down, or not supported by this build
                pass
        prefix = dist.PrefixStore(f"comm-epoch{self.epoch}-{','.join(map(str, live))}/", self.store)
        tmo = datetime.timedelta(seconds=self.timeout_s)
        if self.backend == "nccl":
            opts = dist.ProcessGroupNCCL.Options()
            opts._timeout = tmo
            pg = dist.ProcessGroupNCCL(prefix, live.index(self.rank), len(live), opts)
        else:
            pg = dist.ProcessGroupGloo(prefix, live.index(self.rank), len(live), tmo)
        self.pg = pg
        self.members = live

    # ---------------------------------------------------------------- collectives
    def _dev(self):
        return torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" else torch.device("cpu")

    def alltoall(self, out, inp, out_splits, in_splits):
        """``*_splits`` indexed by logical rank; entries of non-members must be 0."""
        osp = [int(out_splits[r]) for r in self.members]
        isp = [int(in_splits[r]) for r in self.members]
        if sum(osp) != sum(out_splits) or sum(isp) != sum(in_splits):
            raise RuntimeError("traffic addressed to a rank that is not a member")
        self._wait(self.pg.alltoall_base(out, inp, osp, isp, dist.AllToAllOptions()), block=False)

    def alltoall_counts(self, counts):
        """counts[r] = list of k ints for logical rank r -> received[r] (k ints each)."""
        k = len(counts[0]) if counts else 0
        m = len(self.members)
        t = torch.tensor([v for r in self.members for v in counts[r]], dtype=torch.int64, device=self._dev())
        o = torch.empty_like(t)
        self._wait(self.pg.alltoall_base(o, t, [k] * m, [k] * m, dist.AllToAllOptions()))
        vals = o.view(m, k).cpu().tolist()
        out = [[0] * k for _ in range(self.world)]
        for i, r in enumerate(self.members):
            out[r] = vals[i]
        return out

    def allgather_bytes(self, data: bytes):
        """Variable-size all-gather -> {logical rank: bytes}."""
        dev = self._dev()
        m = len(self.members)
        n = torch.tensor([len(data)], dtype=torch.int64, device=dev)
        ns = [torch.empty(1, dtype=torch.int64, device=dev) for _ in range(m)]
        self._wait(self.pg.allgather([ns], [n]))
        sizes = [int(x.item()) for x in ns]
        cap = max(sizes) if sizes else 0
        buf = torch.zeros(max(cap, 1), dtype=torch.uint8, device=dev)
        if data:
            buf[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
        outs = [torch.empty(max(cap, 1), dtype=torch.uint8, device=dev) for _ in range(m)]
        self._wait(self.pg.allgather([outs], [buf]))
        return {r: outs[i][:sizes[i]].cpu().numpy().tobytes() for i, r in enumerate(self.members)}

    def alltoall_bytes(self, out):
        """Variable-size all-to-all: ``out`` = {logical rank: bytes} -> {logical rank: bytes}
        received from each live member (the host side of X2/X3, parallel/links.py)."""
        m = len(self.members)
        sizes = [[len(out.get(r, b""))] for r in range(self.world)]
        got = self.alltoall_counts(sizes)
        osz = [len(out.get(r, b"")) for r in self.members]
        isz = [got[r][0] for r in self.members]
        dev = self._dev()
        flat = b"".join(out.get(r, b"") for r in self.members)
        inp = torch.frombuffer(bytearray(flat or b"\0"), dtype=torch.uint8)[:len(flat)].to(dev)
        o = torch.empty(sum(isz), dtype=torch.uint8, device=dev)
        self._wait(self.pg.alltoall_base(o, inp, isz, osz, dist.AllToAllOptions()))   # every member calls it
        data = o.cpu().numpy().tobytes()
        res, pos = {}, 0
        for i, r in enumerate(self.members):
            res[r] = data[pos:pos + isz[i]]
            pos += isz[i]
        return res

    def allgather_json(self, obj):
        got = self.allgather_bytes(json.dumps(obj).encode())
        return {r: json.loads(b.decode()) for r, b in got.items()}

    def barrier(self):
        self.allgather_bytes(b"")
