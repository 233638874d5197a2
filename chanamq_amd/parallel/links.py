"""Remote consumption across ranks: a consumer on any rank for a queue
owned by another.

The reference lets a consumer on any node pull from any queue: the QueueEntity (owner)
pushes deliveries to the consumer's FrameStage on another node and acks / requeues go
back to the entity (FrameStage.scala:395-429, QueueEntity.scala:318-446).  Here a
*link* joins the two ranks:

* owner side (rank A, owns queue Q): a pseudo connection holding one manual-ack consumer
  on Q with the remote consumer's prefetch.  A's own ``k_dequeue`` serves it (credit,
  round-robin with A's local consumers, TTL skip) and assigns *A's* delivery tags; the
  unacked window of that pseudo channel is the owner's record of what the remote
  consumer holds (X2a credits = that window).
* connection side (rank B): a shadow queue ``amq.link.<id>`` placed on B, into which the
  owner's deliveries are restored (bodies, properties, exchange / routing key and the
  redelivered bit preserved; the message id carries A's tag).  The client's consumer is a
  plain local consumer of the shadow queue, so B assigns the client's delivery tags,
  renders Basic.Deliver at the client's frame-max and enforces its prefetch (X2b).
* acks (X3): consumption of a shadow message on B (ack, auto-ack) is reported by B's
  data plane like a durable-queue consumed record (the shadow is marked durable and its
  messages persistent) and sent back to A, which acks the matching tag on the pseudo
  channel.  Nack / reject with requeue on B put the message back at the head of the
  shadow (redelivered to the same consumer); cancel / channel close / connection close
  close the link: A closes the pseudo channel, so everything the remote consumer still
  held goes back to Q flagged redelivered, and B drops the shadow.

Basic.Get of a queue another rank owns rides a *get link* (``get=True``): the owner side
is a pseudo channel without a consumer, and each Get on rank B is a replicated
``link_pull`` op; when it is applied the owner runs Basic.Get on its queue for the pseudo
channel (manual ack, so the message stays the owner's until B's client acks it) and sends
the message — or "empty" — with the owner's remaining count back to B, which restores it
into the get link's shadow and answers the client with a local Basic.Get on the shadow
(reference: Basic.Get pulls one message from the QueueEntity on whatever node owns it,
FrameStage.scala:1199-1229, QueueEntity.scala:318-393).

The per-step traffic (owner -> consumer deliveries, consumer -> owner acks) is one
variable-size all-to-all between the live ranks after the data step (``Comm.alltoall_bytes``,
or local copies in ``LocalCluster``); it runs only while links exist, and every rank
knows that from the replicated control log.
"""

import struct

from ..engine.control import ControlError, C

LINK_PREFIX = "amq.link."
_EPOCH_SHIFT = 40
K_DELIVER, K_ACK, K_GOT, K_EMPTY = 1, 2, 3, 4
_HDR = ">BIIQBBBII"          # kind, link, epoch, tag, redelivered, |ex|, |rk|, |props|, |body|


class Link:
    __slots__ = ("id", "vhost", "queue", "dest", "prefetch", "shadow", "epoch", "pc", "closing", "get",
                 "pending", "slot")

    def __init__(self, lid, vhost, queue, dest, prefetch, get=False):
        self.id, self.vhost, self.queue, self.dest, self.prefetch = lid, vhost, queue, dest, prefetch
        self.shadow = LINK_PREFIX + str(lid)
        self.epoch, self.pc, self.closing, self.get = 0, None, False, bool(get)
        self.pending = set()     # connection side of a get link: pulls not answered yet
        self.slot = None         # shadow queue slot (device links)


def parse_delivers(buf):
    """Basic.Deliver + content frames -> [(tag, redelivered, exchange, routing_key,
    raw properties, body)]."""
    out, pos, n = [], 0, len(buf)
    cur = None
    while pos + 7 <= n:
        t, _, size = struct.unpack_from(">BHI", buf, pos)
        p = pos + 7
        if t == 1:
            cls, mid = struct.unpack_from(">HH", buf, p)
            if cls == 60 and mid == 60:
                q = p + 4
                q += 1 + buf[q]                                  # consumer tag
                tag = struct.unpack_from(">Q", buf, q)[0]
                red = bool(buf[q + 8] & 1)
                q += 9
                ex = bytes(buf[q + 1:q + 1 + buf[q]])
                q += 1 + buf[q]
                rk = bytes(buf[q + 1:q + 1 + buf[q]])
                cur = [tag, red, ex, rk, b"", bytearray(), 0]
        elif t == 2 and cur is not None:
            cur[6] = struct.unpack_from(">Q", buf, p + 4)[0]
            cur[4] = bytes(buf[p + 12:p + size])
            if cur[6] == 0:
                out.append(tuple(cur[:5]) + (b"",))
                cur = None
        elif t == 3 and cur is not None:
            cur[5] += buf[p:p + size]
            if len(cur[5]) >= cur[6]:
                out.append(tuple(cur[:5]) + (bytes(cur[5]),))
                cur = None
        pos = p + size + 1
    return out


def parse_get_ok(buf):
    """Basic.GetOk + content frames -> (tag, redelivered, exchange, routing_key, raw
    properties, body, message_count)."""
    p = 7 + 4
    tag = struct.unpack_from(">Q", buf, p)[0]
    red = bool(buf[p + 8] & 1)
    q = p + 9
    ex = bytes(buf[q + 1:q + 1 + buf[q]])
    q += 1 + buf[q]
    rk = bytes(buf[q + 1:q + 1 + buf[q]])
    q += 1 + buf[q]
    cnt = struct.unpack_from(">I", buf, q)[0]
    pos = 7 + struct.unpack_from(">I", buf, 3)[0] + 1
    size = struct.unpack_from(">I", buf, pos + 3)[0]
    blen = struct.unpack_from(">Q", buf, pos + 7 + 4)[0]
    props = bytes(buf[pos + 7 + 12:pos + 7 + size])
    pos += 7 + size + 1
    body = bytearray()
    while len(body) < blen and pos + 7 <= len(buf):
        size = struct.unpack_from(">I", buf, pos + 3)[0]
        body += buf[pos + 7:pos + 7 + size]
        pos += 7 + size + 1
    return tag, red, ex, rk, props, bytes(body), cnt


def set_get_ok_count(frames, count):
    """The message-count field of a rendered Basic.GetOk (the first frame of ``frames``)."""
    b = bytearray(frames)
    q = 7 + 4 + 9
    q += 1 + b[q]
    q += 1 + b[q]
    struct.pack_into(">I", b, q, int(count))
    return bytes(b)


class RemoteLinks:
    """Links of one rank (one per plane).  ``alloc_conn`` / ``free_conn`` hand out the
    pseudo-connection slots (the server passes its connection-slot allocator)."""

    def __init__(self, plane, alloc_conn=None, free_conn=None):
        self.plane = plane
        self.links = {}          # id -> Link (replicated: every rank knows every link)
        self.by_shadow = {}      # shadow queue slot -> Link (connection side)
        self._restore = []       # received deliveries, restored before the next step
        self._next_pc = plane.c_max - 2
        self._pulled = {}        # owner side of get links: dest rank -> records of this step
        self.got = []            # connection side: answered pulls [(pull id, link id, count | None)]
        self._alloc = alloc_conn or self._default_alloc
        self._free = free_conn or (lambda c: None)

    def _default_alloc(self):
        while self._next_pc > 0 and self._next_pc in self.plane.conns:
            self._next_pc -= 1
        if self._next_pc <= 0:
            raise ControlError(C.RESOURCE_ERROR, "no connection slot for a link", 60, 20)
        c, self._next_pc = self._next_pc, self._next_pc - 1
        return c

    @property
    def active(self):
        return bool(self.links)

    # ------------------------------------------------------------------ control ops
    def open(self, lid, vhost, queue, dest, prefetch=0, get=False):
        """Replicated (control log ``link_open``): applied in the same order on every rank."""
        p = self.plane
        q = p.queues.get((vhost, queue))
        if q is None:
            raise ControlError(C.NOT_FOUND, f"no queue '{queue}' in vhost '{vhost}'", 60, 20)
        if dest == p.rank and hasattr(p, "eng") and not p.info.get("persist"):
            raise ControlError(C.NOT_IMPLEMENTED, "remote consumers need the engine built with persist=1", 60, 20)
        lk = Link(lid, vhost, queue, dest, int(prefetch) or 1024, get)
        p.shard_map.place(vhost, lk.shadow, dest)
        slot = p.declare_queue(vhost, lk.shadow, durable=True)
        self.links[lid] = lk
        if dest == p.rank:
            self.by_shadow[slot] = lk
            if hasattr(p, "link_slots"):
                p.link_slots.add(slot)
        if q.owner == p.rank:
            self._attach(lk)
        return slot

    def _attach(self, lk):
        """Owner side: the pseudo consumer on the source queue (a fresh epoch: tags
        restart with the new pseudo channel)."""
        p = self.plane
        pc = self._alloc()
        p.open_connection(pc, lk.vhost)
        p.open_channel(pc, 1)
        if not lk.get:
            p.qos(pc, 1, prefetch_count=lk.prefetch)
            p.consume(pc, 1, lk.vhost, lk.queue, "amq.link-" + str(lk.id), no_ack=False)
        lk.pc, lk.epoch = pc, lk.epoch + 1

    def _detach(self, lk):
        if lk.pc is not None:
            self.plane.close_connection(lk.pc)   # unacked -> back to the queue, redelivered
            self._free(lk.pc)
            lk.pc = None

    def close(self, lid):
        """Replicated (``link_close``).  The owner keeps the pseudo channel until the
        step's acks came back (``after_step``); the connection side purges the shadow now
        and deletes it after the next step released the purged entries."""
        lk = self.links.get(lid)
        if lk is None or lk.closing:
            return None
        lk.closing = True
        sq = self.plane.queues.get((lk.vhost, lk.shadow))
        if sq is not None and sq.owner == self.plane.rank:
            self.plane.purge(sq.slot)
        return None

    def pull(self, lid, pn, now_ms=None):
        """Replicated (``link_pull``): one Basic.Get for get link ``lid``, pull id ``pn``.
        The owner takes the head of the queue for its pseudo channel now (between steps)
        and answers after the step (``outgoing``).  Returns False when the link is gone
        (the connection side then answers Get-Empty itself)."""
        lk = self.links.get(lid)
        if lk is None or lk.closing or not lk.get:
            return False
        if lk.dest == self.plane.rank:
            lk.pending.add(pn)
        if lk.pc is None:   # owner side not attached here
            return True
        p = self.plane
        q = p.queues.get((lk.vhost, lk.queue))
        rec = self._pulled.setdefault(lk.dest, bytearray())
        frames, cnt = None, 0
        if q is not None and q.owner == p.rank:
            try:
                frames, cnt = (p.basic_get(lk.pc, 1, q.slot, False, now_ms) if now_ms is not None
                               else p.basic_get(lk.pc, 1, q.slot, False))
            except ControlError:   # the pseudo channel's delivery window is full
                frames = None
        if frames is None:
            rec += struct.pack(">BIQI", K_EMPTY, lid, pn, cnt)
        else:
            tag, red, ex, rk, props, body, cnt = parse_get_ok(frames)
            rec += struct.pack(_HDR + "QI", K_GOT, lid, lk.epoch, tag, int(red), len(ex), len(rk), len(props),
                               len(body), pn, cnt) + ex + rk + props + body
        return True

    def take_gets(self):
        """Connection side: answered pulls since the last call, [(pull id, link id, owner's
        remaining count, or None for empty)]; the messages are in the shadows once
        ``before_step`` ran."""
        out, self.got = self.got, []
        return out

    def shadow_of(self, lid):
        lk = self.links.get(lid)
        return lk.shadow if lk else None

    # ------------------------------------------------------------------ per step
    def before_step(self, now_ms=None):
        """Deliveries the last exchange brought go into the shadow queues (connection
        side).  Deferred to just before the next step: a GPU restore is a small step of its
        own and would overwrite the host-visible records the server still reads."""
        p = self.plane
        items, self._restore = self._restore, []
        if items:
            p.restore(items, now_ms) if now_ms is not None else p.restore(items)

    def outgoing(self, eg):
        """After the data step: {dest rank: bytes}.  Takes the pseudo connections' bytes
        out of the step's egress {conn: bytes} (no socket behind them)."""
        p = self.plane
        out, self._pulled = self._pulled, {}
        for lk in self.links.values():
            if lk.pc is None or lk.get:
                continue
            buf = eg.pop(lk.pc, None)
            if not buf:
                continue
            b = out.setdefault(lk.dest, bytearray())
            for tag, red, ex, rk, props, body in parse_delivers(buf):
                b += struct.pack(_HDR, K_DELIVER, lk.id, lk.epoch, tag, int(red), len(ex), len(rk),
                                 len(props), len(body)) + ex + rk + props + body
        if self.by_shadow:
            for mid, q, _qpos, kind in p.take_link_consumed(self.by_shadow):
                lk = self.by_shadow[q]
                if kind != 0:   # only consumption is reported; requeues stay in the shadow
                    continue
                owner = p.queues[(lk.vhost, lk.queue)].owner
                out.setdefault(owner, bytearray()).extend(
                    struct.pack(">BIIQ", K_ACK, lk.id, mid >> _EPOCH_SHIFT, mid & ((1 << _EPOCH_SHIFT) - 1)))
        return {r: bytes(b) for r, b in out.items()}

    def incoming(self, got):
        """Records from every rank -> pending acks / restores (applied by ``before_step``)."""
        p = self.plane
        for src in sorted(got):
            buf, pos = got[src], 0
            while pos < len(buf):
                k = buf[pos]
                if k == K_ACK:   # owner side: ack the tag on the pseudo channel now (before
                    _, lid, epoch, tag = struct.unpack_from(">BIIQ", buf, pos)   # a closing link
                    pos += 17                                                     # is detached)
                    lk = self.links.get(lid)
                    if lk is not None and lk.pc is not None and lk.epoch == epoch:
                        p.apply_ack(lk.pc, 1, tag)
                    continue
                if k == K_EMPTY:   # connection side: the owner's queue was empty
                    _, lid, pn, cnt = struct.unpack_from(">BIQI", buf, pos)
                    pos += 17
                    self._answered(lid, pn, None)
                    continue
                _, lid, epoch, tag, red, lex, lrk, lp, lb = struct.unpack_from(_HDR, buf, pos)
                pos += 28
                if k == K_GOT:
                    pn, cnt = struct.unpack_from(">QI", buf, pos)
                    pos += 12
                ex = buf[pos:pos + lex]
                pos += lex
                rk = buf[pos:pos + lrk]
                pos += lrk
                props = buf[pos:pos + lp]
                pos += lp
                body = buf[pos:pos + lb]
                pos += lb
                lk = self.links.get(lid)
                sq = p.queues.get((lk.vhost, lk.shadow)) if lk is not None and not lk.closing else None
                if k == K_GOT:
                    self._answered(lid, pn, cnt if sq is not None else None)
                if sq is None:
                    continue   # the owner requeued it when the link closed
                self._restore.append((sq.slot, (epoch << _EPOCH_SHIFT) | tag, 0, 0, bytes(ex), bytes(rk),
                                      bytes(props), bytes(body), True, bool(red)))

    def _answered(self, lid, pn, cnt):
        lk = self.links.get(lid)
        if lk is not None:
            lk.pending.discard(pn)
        self.got.append((pn, lid, cnt))

    def after_step(self):
        """Finish closing links: the owner closes the pseudo channel (after this step's
        acks were applied), the connection side deletes the drained shadow."""
        p = self.plane
        for lid in [l for l, lk in self.links.items() if lk.closing]:
            lk = self.links.pop(lid)
            self._detach(lk)
            sq = p.queues.get((lk.vhost, lk.shadow))
            if sq is not None:
                self.by_shadow.pop(sq.slot, None)
                getattr(p, "link_slots", set()).discard(sq.slot)
                p.delete_queue(lk.vhost, lk.shadow)
            p.shard_map.placement.pop(_eid(lk.vhost, lk.shadow), None)

    # ------------------------------------------------------------------ failover
    def on_failure(self, dead):
        """Before the queues are re-homed: links whose consumer side died close (their
        shadows go; the owner requeues what they held); links whose owner died lose the
        pseudo channel (its window was on the dead GPU) and re-attach at the queue's new
        owner after ``rehome`` (``after_rehome``)."""
        p = self.plane
        self.lost_owner(dead)
        for lid in [l for l, lk in self.links.items() if lk.dest in dead]:
            lk = self.links.pop(lid)
            self._detach(lk)
            sq = p.queues.get((lk.vhost, lk.shadow))
            if sq is not None:
                self.by_shadow.pop(sq.slot, None)
                getattr(p, "link_slots", set()).discard(sq.slot)
                p.delete_queue(lk.vhost, lk.shadow)
            p.shard_map.placement.pop(_eid(lk.vhost, lk.shadow), None)

    def lost_owner(self, dead):
        """Connection side of get links whose queue owner died: their outstanding pulls
        will not be answered by it (``on_failure`` runs before the re-home)."""
        p = self.plane
        for lk in self.links.values():
            q = p.queues.get((lk.vhost, lk.queue))
            if lk.get and lk.pending and q is not None and q.owner in dead:
                for pn in sorted(lk.pending):
                    self.got.append((pn, lk.id, None))
                lk.pending.clear()

    def after_rehome(self):
        p = self.plane
        for lk in self.links.values():
            q = p.queues.get((lk.vhost, lk.queue))
            if q is not None and q.owner == p.rank and lk.pc is None and not lk.closing:
                self._attach(lk)


def _eid(vhost, name):
    from ..engine.control import entity_id
    return entity_id(vhost, name)


class DeviceLinks:
    """Remote consumers on the device (the pipelined sharded server, X2/X3).

    Same link model as ``RemoteLinks`` -- owner-side pseudo connection + consumer on the
    source queue, connection-side shadow queue holding the owner's deliveries, acks back
    to the owner -- but the per-message traffic never reaches the host: the owner's
    ``k_render`` turns the pseudo connection's deliveries into restore records (RDesc,
    MF_RESTORE into the shadow, redelivered bit, id = epoch << 40 | owner tag) that ride
    the next per-step exchange with the publishes; the connection side's data plane turns
    every consumption of a shadow message into an ack record for the owner, whose phase B
    marks the tag acked in the pseudo channel (``k_link_acks``).  Link open / close run at
    the control syncs (every rank applies them at the same step, nothing in flight).

    Basic.Get of a remote queue (get link): the owner runs Basic.Get on its pseudo
    channel at the sync that applies the ``link_pull`` and answers with a replicated
    ``link_got`` op; the connection side restores the message into the get link's shadow
    at the next sync.  Reference: FrameStage.scala:395-429 / 1199-1229,
    QueueEntity.scala:318-446.
    """

    def __init__(self, plane, alloc_conn, free_conn, submit):
        self.plane = plane
        self.links = {}
        self._alloc, self._free, self._submit = alloc_conn, free_conn, submit
        self.got = []             # connection side: answered pulls [(pull id, link id, count | None)]
        self._link_conns = []     # owner side: pseudo connections (device list, <= 64)

    @property
    def active(self):
        return bool(self.links)

    def shadow_of(self, lid):
        lk = self.links.get(lid)
        return lk.shadow if lk else None

    def before_step(self, now_ms=None):
        """Device links restore nothing between steps (records arrive with the exchange)."""

    def take_gets(self):
        out, self.got = self.got, []
        return out

    def _sync_conns(self):
        self.plane.set_link_conns(self._link_conns)

    # ------------------------------------------------------------------ replicated ops
    def open(self, lid, vhost, queue, dest, prefetch=0, get=False):
        p = self.plane
        q = p.queues.get((vhost, queue))
        if q is None:
            raise ControlError(C.NOT_FOUND, f"no queue '{queue}' in vhost '{vhost}'", 60, 20)
        if len(self._link_conns) >= 64 and q.owner == p.rank:
            raise ControlError(C.RESOURCE_ERROR, "too many remote-consumer links on this rank", 60, 20)
        lk = Link(lid, vhost, queue, dest, int(prefetch) or 1024, get)
        p.shard_map.place(vhost, lk.shadow, dest)
        slot = p.declare_queue(vhost, lk.shadow)
        lk.slot = slot
        self.links[lid] = lk
        if dest == p.rank:
            p.set_link_queue(slot, q.owner)   # consumption here -> acks to the owner
        if q.owner == p.rank:
            self._attach(lk)
        return slot

    def _attach(self, lk):
        p = self.plane
        pc = self._alloc()
        p.open_connection(pc, lk.vhost)
        p.open_channel(pc, 1)
        if not lk.get:
            p.qos(pc, 1, prefetch_count=lk.prefetch)
            p.consume(pc, 1, lk.vhost, lk.queue, "amq.link-" + str(lk.id), no_ack=False)
        lk.pc, lk.epoch = pc, lk.epoch + 1
        p.set_link_conn(pc, lk.dest, lk.slot, lk.epoch)
        self._link_conns.append(pc)
        self._sync_conns()

    def _detach(self, lk):
        """Owner side: the pseudo channel closes -- what the remote consumer still held goes
        back to the queue, redelivered (its requeue settles in the next step)."""
        p = self.plane
        if lk.pc is not None:
            p.clear_link_conn(lk.pc, lk.slot)
            if lk.pc in self._link_conns:
                self._link_conns.remove(lk.pc)
            self._sync_conns()
            p.close_connection(lk.pc)
            p.step({})            # settle the requeue before the slot can be reused
            self._free(lk.pc)
            lk.pc = None

    def _drop_shadow(self, lk):
        p = self.plane
        sq = p.queues.get((lk.vhost, lk.shadow))
        if sq is not None:
            if sq.owner == p.rank:
                p.set_link_queue(sq.slot, None)
                left = p.purge(sq.slot)
                while left:   # release the purged entries (no acks any more)
                    p.step({})
                    now = p.message_count(sq.slot)
                    if now >= left:
                        break
                    left = now
            p.delete_queue(lk.vhost, lk.shadow)
        p.shard_map.placement.pop(_eid(lk.vhost, lk.shadow), None)

    def close(self, lid):
        lk = self.links.pop(lid, None)
        if lk is None:
            return None
        lk.closing = True
        self._detach(lk)
        self._drop_shadow(lk)
        for pn in sorted(lk.pending):   # unanswered Gets of a closed get link: empty
            self.got.append((pn, lk.id, None))
        return None

    def pull(self, lid, pn, now_ms=None):
        lk = self.links.get(lid)
        if lk is None or lk.closing or not lk.get:
            return False
        p = self.plane
        if lk.dest == p.rank:
            lk.pending.add(pn)
        if lk.pc is None:
            return True
        q = p.queues.get((lk.vhost, lk.queue))
        frames, cnt = None, 0
        if q is not None and q.owner == p.rank:
            try:
                frames, cnt = p.basic_get(lk.pc, 1, q.slot, False)
            except ControlError:   # the pseudo channel's window is full
                frames = None
        if frames is None:
            self._submit("link_got", lid, pn, None)
        else:
            tag, red, ex, rk, props, body, cnt = parse_get_ok(frames)
            self._submit("link_got", lid, pn, [cnt, lk.epoch, tag, int(red), ex.hex(), rk.hex(), props.hex(),
                                               body.hex()])
        return True

    def got_answer(self, lid, pn, ans):
        """Replicated ``link_got``: the connection side restores the message into the get
        link's shadow queue (at this sync point) and records the answer."""
        lk = self.links.get(lid)
        p = self.plane
        if lk is None or lk.dest != p.rank:
            return None
        lk.pending.discard(pn)
        sq = p.queues.get((lk.vhost, lk.shadow))
        if ans is None or sq is None:
            self.got.append((pn, lid, None))
            return None
        cnt, epoch, tag, red, ex, rk, props, body = ans
        p.restore([(sq.slot, (int(epoch) << _EPOCH_SHIFT) | int(tag), 0, 0, bytes.fromhex(ex), bytes.fromhex(rk),
                    bytes.fromhex(props), bytes.fromhex(body), False, bool(red))])
        self.got.append((pn, lid, int(cnt)))
        return None

    # ------------------------------------------------------------------ failover
    def on_failure(self, dead):
        p = self.plane
        for lk in list(self.links.values()):
            q = p.queues.get((lk.vhost, lk.queue))
            if lk.get and lk.pending and q is not None and q.owner in dead:
                for pn in sorted(lk.pending):
                    self.got.append((pn, lk.id, None))
                lk.pending.clear()
            if lk.dest in dead:   # the consumer side is gone: the owner requeues what it held
                self.links.pop(lk.id)
                self._detach(lk)
                self._drop_shadow(lk)

    def after_rehome(self):
        """Links whose queue moved here re-attach (a new epoch: acks of deliveries made by
        the dead owner are ignored); connection sides point their acks at the new owner."""
        p = self.plane
        for lk in self.links.values():
            q = p.queues.get((lk.vhost, lk.queue))
            if q is None:
                continue
            if lk.dest == p.rank:
                p.set_link_queue(lk.slot, q.owner)
            if q.owner == p.rank and lk.pc is None and not lk.closing:
                self._attach(lk)
