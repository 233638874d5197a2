"""In-process sharded cluster: W data planes (GPU or golden) stepped in lockstep, the
cross-rank exchange done by local copies.  Used by tests on one device and as the
reference for the one-process-per-GPU deployment (each rank then owns one plane and an
``Exchanger`` over RCCL).  Control operations are replicated to every plane in the same
order so queue/exchange slots agree across ranks."""

from .exchange import local_exchange
from .links import RemoteLinks
from .shard import ShardMap


class LocalCluster:
    def __init__(self, make_plane, world, shard_map=None):
        self.world = world
        self.shard_map = shard_map or ShardMap(world)
        self.planes = [make_plane(rank=r, world=world, shard_map=self.shard_map) for r in range(world)]
        self.links = [RemoteLinks(p) for p in self.planes]

    def __getitem__(self, r):
        return self.planes[r]

    def replicate(self, fn, *args, **kw):
        """Apply a control-plane op (declare/bind/delete ...) on every rank."""
        return [getattr(p, fn)(*args, **kw) for p in self.planes]

    def link_open(self, lid, vhost, queue, dest, prefetch=0, get=False):
        """Remote consumer link (parallel/links.py), replicated like a control op;
        returns the shadow queue's name (consume it on rank ``dest``; a get link's shadow
        receives the messages its pulls fetched)."""
        for lk in self.links:
            lk.open(lid, vhost, queue, dest, prefetch, get)
        return self.links[0].shadow_of(lid)

    def link_pull(self, lid, pn, now_ms=None):
        """One remote Basic.Get on get link ``lid`` (answered after the next step)."""
        return [lk.pull(lid, pn, now_ms) for lk in self.links][0]

    def link_close(self, lid):
        for lk in self.links:
            lk.close(lid)

    def step(self, inputs_by_rank, now_ms=0):
        """``inputs_by_rank``: [ {conn: bytes} per rank ] -> [StepResult/dict per rank]."""
        gpu = hasattr(self.planes[0], "eng")
        for lk in self.links:
            lk.before_step()
        tickets = []
        for r, p in enumerate(self.planes):
            inp = inputs_by_rank[r] if r < len(inputs_by_rank) else {}
            if gpu:
                tickets.append(_gpu_submit(p, inp, now_ms))
            else:
                p.step_a(inp, now_ms)
        recv = local_exchange(self.planes)
        out = []
        for r, p in enumerate(self.planes):
            if gpu:
                if p.lag:   # phase B already ran (importing the previous exchange)
                    p.set_import(recv[r])
                else:
                    p.submit_b(recv[r])
                out.append(p.finish(tickets[r]))
            else:
                out.append(p.step_b(recv[r]))
        if self.links[0].active:   # X2/X3 link traffic, local copies
            sent = [lk.outgoing(o["egress"] if isinstance(o, dict) else o.egress) for lk, o in zip(self.links, out)]
            for r, lk in enumerate(self.links):
                lk.incoming({s: sent[s].get(r, b"") for s in range(self.world)})
            for lk in self.links:
                lk.after_step()
        return out


def _gpu_submit(plane, inputs, now_ms):
    """GpuDataPlane.step() without the collective: stage ingress and run phase A."""
    segs, ptr, n = plane.stage(inputs)
    return plane.submit_raw(segs, ptr, n, now_ms)
