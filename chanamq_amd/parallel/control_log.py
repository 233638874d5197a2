"""Replicated control plane (the role of the reference's DistributedPubSub broadcasts
and entity messages for exchange/queue/binding changes).

Control operations issued on any rank are appended to that rank's outbox; ``sync()``
all-gathers the outboxes once per step and every rank applies the union in the same
order (logical rank, then sequence), so the replicated tables (exchanges, bindings,
queue slots, ownership) stay identical everywhere.  Connection-scoped state (channels,
consumers) stays local and is not logged.  Ops are JSON: nothing executable crosses
ranks.
"""

from ..protocol import constants as C
from .comm import Comm

REPLICATED = {"declare_exchange", "delete_exchange", "declare_queue", "delete_queue", "bind", "unbind",
              "place_queue", "ensure_vhost", "link_open", "link_close", "link_pull", "link_got", "big_publish"}


class ControlLog:
    def __init__(self, plane, comm: Comm):
        self.plane, self.comm = plane, comm
        self.outbox = []
        self.blobs = {}       # local seq -> (bytes, destination ranks): bulk payload of an op
        self.applied = 0
        self.results = {}     # local seq -> result or ControlError tuple
        self.handlers = {}    # op -> callable for ops served above the plane (parallel/links.py)
        self.on_applied = None   # (op, args, kw, result) after each applied op (store rows)

    def submit(self, op, *args, blob=None, blob_to=(), **kw):
        """``blob`` (bytes) travels only to the ranks ``blob_to`` -- one variable-size
        all-to-all at the sync, not inside the all-gathered JSON -- and reaches the op's
        handler there as ``blob=`` (None on the other ranks)."""
        if op not in REPLICATED:
            raise ValueError(f"{op} is not a replicated control op")
        seq = len(self.outbox)
        self.outbox.append([op, list(args), kw])
        if blob is not None:
            self.blobs[seq] = (bytes(blob), sorted({int(r) for r in blob_to}))
        return seq

    def _pack_blobs(self, batch, blobs):
        """Per destination rank, the concatenated blobs of this batch; each op with a blob
        records {dest: [offset, length]} in its kw (``_blob``)."""
        out = {}
        for seq, (data, dests) in blobs.items():
            where = {}
            for r in dests:
                buf = out.setdefault(r, bytearray())
                where[str(r)] = [len(buf), len(data)]
                buf += data
            batch[seq][2] = dict(batch[seq][2], _blob=where)
        return {r: bytes(b) for r, b in out.items()}

    def sync(self):
        """All-gather and apply.  Returns {local seq: result} for this rank's ops."""
        from ..engine.control import ControlError
        # ops submitted while this batch is applied (e.g. an owner's link_got answer) go
        # into the next batch
        batch, self.outbox = self.outbox, []
        blobs, self.blobs = self.blobs, {}
        sent = self._pack_blobs(batch, blobs)
        try:
            got = self.comm.allgather_json(batch)
            # every rank sees the same gathered batches, so all of them take part in the
            # blob all-to-all or none does
            recv = {}
            if any("_blob" in kw for r in got for _, _, kw in got[r]):
                recv = self.comm.alltoall_bytes(sent)
        except RuntimeError:
            for seq, b in blobs.items():   # retried after the failover
                self.blobs[seq] = b
                batch[seq][2].pop("_blob", None)
            self.outbox = batch + self.outbox
            raise
        mine = {}
        for r in sorted(got):
            for seq, (op, args, kw) in enumerate(got[r]):
                if "_blob" in kw:
                    kw = dict(kw)
                    where = kw.pop("_blob").get(str(self.comm.rank))
                    kw["blob"] = recv.get(r, b"")[where[0]:where[0] + where[1]] if where else None
                try:
                    res = self._apply(op, args, kw)
                except ControlError as e:
                    res = ("error", e.code, e.text, e.class_id, e.method_id)
                except Exception as e:   # a failing op must not read as a lost peer (_retry)
                    import logging
                    logging.getLogger("chanamq.control").exception("control op %s failed", op)
                    res = ("error", C.INTERNAL_ERROR, f"{op}: {e}"[:255], 0, 0)
                if self.on_applied is not None:
                    self.on_applied(op, args, kw, res)
                self.applied += 1
                if r == self.comm.rank:
                    mine[seq] = res
        return mine

    def _apply(self, op, args, kw):
        p = self.plane
        if op in self.handlers:
            return self.handlers[op](*args, **kw)
        if op == "place_queue":
            vhost, name, rank = args
            q = p.queues.get((vhost, name))
            if q is None:
                p.shard_map.place(vhost, name, rank)
                return None
            p.shard_map.place(vhost, name, rank)
            return p.set_queue_owner(q.slot, rank)
        if op == "ensure_vhost":
            return p.ensure_vhost(*args)
        return getattr(p, op)(*args, **kw)


def error_of(res):
    """(code, text, class, method) if ``res`` is a logged ControlError, else None."""
    if isinstance(res, (list, tuple)) and res and res[0] == "error":
        return tuple(res[1:])
    return None


__all__ = ["ControlLog", "error_of", "REPLICATED", "C"]
