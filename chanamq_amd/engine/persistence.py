"""Write-behind persistence for the GPU data plane (SURVEY §3.3, P7 / BASELINE config 4).

Each step the device emits (a) one persist record per enqueue of a persistent message
into a durable queue, packed with the message bytes, and (b) one consumed record per
persistent message that leaves a durable queue (acked, auto-acked, expired).  ``after_step``
turns them into rows of the Cassandra-schema store (csrc/core/store.cpp, same tables
as the reference's create-cassantra.cql):

  msgs(id, tstamp, header, body, exchange, routing, durable, refer)   once per message
  queues(queue, offset, msgid, size)                                   per durable queue
  -> deleted when consumed; the message row when its refer count drops to zero

and the server calls ``commit()`` (one fsync, group commit) before it releases the
step's egress, so a publisher confirm is never sent before its message is durable.

``recover`` rebuilds durable vhosts/exchanges/queues/bindings from the store and feeds
the stored messages back through the device import path (``restore``) — unacked ones
first, flagged redelivered (reference QueueEntity.scala:117 never requeued them: A.Q31).
Queue offsets restart at 0 on the device, so recovery rewrites the queue rows to the new
offsets in the same commit.
"""

import struct

from .control import entity_id

LINK_SHADOW = "amq.link."   # shadow queues of cross-rank links (parallel/links.py): never stored


def _split_eid(eid):
    if "-_." in eid:
        v, n = eid.split("-_.", 1)
        return v, n
    return "", eid


class GpuPersistence:
    def __init__(self, plane, store):
        self.plane, self.store = plane, store
        self.refs = {}            # msg id -> durable queue rows referencing it
        self.rows = {}            # (queue id, msg id) -> [stored offset, size, is_unack]
        self.rows_written = 0
        self.dirty = False
        self.native = None        # PersistWorker (csrc/core/persist.cpp) once attached

    def attach_native(self, worker):
        """Hand the row bookkeeping to the native write-behind worker (pipelined front
        end): from now on every record goes through it, Python keeps only control rows."""
        self.native = worker
        for q in self.plane.queue_by_slot.values():
            if q.durable and not q.name.startswith(LINK_SHADOW):
                worker.set_queue(q.slot, entity_id(q.vhost, q.name))
        for (qid, mid), (off, size, unack) in self.rows.items():
            worker.seed_row(qid, mid, off, size, bool(unack), self.refs.get(mid, 1))
        self.rows, self.refs = {}, {}
        worker.start()

    def submit_raw(self, persist=b"", consumed=b""):
        """Native mode: records of a host-run step / Basic.Get, applied and committed
        before the caller sends that step's egress."""
        if persist or consumed:
            self.native.submit(0, persist, consumed)
            self.native.drain()

    def _qid(self, slot):
        q = self.plane.queue_by_slot.get(slot)
        return entity_id(q.vhost, q.name) if q is not None else None

    # ------------------------------------------------------------------ step records
    def after_step(self):
        """Apply the step's records.  Device queue positions change on requeue, so rows
        are addressed by (queue, message id) -> the offset they were stored at."""
        if self.native is not None:
            from .layout import CONSUMED_REC
            import numpy as np
            persist, consumed = self.plane.take_persist_raw()
            gets = self.plane.take_get_consumed()
            if gets:
                a = np.zeros(len(gets), CONSUMED_REC)
                for i, (mid, q, qpos, kind) in enumerate(gets):
                    a[i] = (mid, qpos, q, kind, (0, 0))
                consumed += a.tobytes()
            self.submit_raw(persist, consumed)
            return bool(persist)
        return self.apply(self.plane.take_persist(), self.plane.take_consumed())

    def apply(self, persisted, consumed):
        """Store rows for a step's persist / consumed records (see after_step)."""
        st = self.store
        for mid, ts, q, qpos, exp, ex, rk, props, body in persisted:
            qid = self._qid(q)
            if qid is None:
                continue
            n = self.refs.get(mid, 0)
            self.refs[mid] = n + 1
            if n == 0:
                header = b"\0\0" + struct.pack(">Q", len(body)) + props
                st.insert_message(mid, ts, header, body, ex.decode("utf-8", "replace"),
                                  rk.decode("utf-8", "replace"), True, 1, 0)
            else:
                st.update_message_refer_count(mid, n + 1)
            st.insert_queue_msg(qid, qpos, mid, len(body), 0)
            self.rows[(qid, mid)] = [qpos, len(body), False]
            self.rows_written += 1
        for mid, q, qpos, kind in consumed:
            qid = self._qid(q)
            row = self.rows.get((qid, mid)) if qid is not None else None
            if row is None:
                continue
            off, size, unack = row
            if kind == 3:                 # delivered, awaiting ack: queues -> queue_unacks
                if not unack:
                    st.insert_queue_unack(qid, off, mid, size)
                    st.delete_queue_msg(qid, off)
                    row[2] = True
                continue
            if kind == 4:                 # requeued: back to queues (redelivered on recovery
                if unack:                 # is implied by the unack history; RabbitMQ-like)
                    st.delete_queue_unack(qid, mid)
                    st.insert_queue_msg(qid, off, mid, size, 0)
                    row[2] = False
                continue
            # consumed / expired / dropped: the row goes, the message when unreferenced
            if unack:
                st.delete_queue_unack(qid, mid)
            else:
                st.delete_queue_msg(qid, off)
            del self.rows[(qid, mid)]
            n = self.refs.get(mid, 1) - 1
            if n <= 0:
                self.refs.pop(mid, None)
                st.delete_message(mid)
            else:
                self.refs[mid] = n
                st.update_message_refer_count(mid, n)
        if persisted or consumed:
            self.dirty = True
        return bool(persisted)

    def commit(self):
        if self.native is not None:
            self.native.drain()
            return
        if self.dirty:
            self.store.sync()
            self.dirty = False

    # ------------------------------------------------------------------ control rows
    def control_commit(self):
        """Topology rows (vhosts, exchanges, queues, bindings) written by the control
        plane reach the disk before the reply: the store buffers WAL records until a sync
        (the write-behind worker syncs only when it has step records)."""
        self.store.sync()

    def vhost(self, name):
        self.store.insert_vhost(name, True)

    def exchange(self, x):
        if x.durable and x.name and not x.name.startswith("amq."):
            self.store.insert_exchange(entity_id(x.vhost, x.name), x.type, True, x.auto_delete, x.internal,
                                       {k: str(v) for k, v in (x.arguments or {}).items()})

    def exchange_deleted(self, vhost, name):
        self.store.delete_exchange(entity_id(vhost, name))

    def queue(self, q):
        if q.durable and not q.name.startswith(LINK_SHADOW):   # link shadows hold no rows
            self.store.insert_queue_meta(entity_id(q.vhost, q.name), -1, set(), True, q.ttl_ms)
            if self.native is not None:
                self.native.set_queue(q.slot, entity_id(q.vhost, q.name))

    def queue_deleted(self, vhost, name, slot=None):
        qid = entity_id(vhost, name)
        if self.native is not None and slot is not None:
            self.native.drain()
            self.native.set_queue(slot, "")
        self.store.force_delete_queue(qid)
        self.store.delete_binds_of_queue(qid)

    def bind(self, vhost, queue, exchange, key):
        x = self.plane.exchanges.get((vhost, exchange))
        q = self.plane.queues.get((vhost, queue))
        if x is not None and q is not None and x.durable and q.durable and exchange and \
                not exchange.startswith("amq."):
            self.store.insert_bind(entity_id(vhost, exchange), entity_id(vhost, queue), key, {})

    def unbind(self, vhost, queue, exchange, key):
        self.store.delete_bind(entity_id(vhost, exchange), entity_id(vhost, queue), key)

    # ------------------------------------------------------------------ failover
    def adopt(self, src, queues, now_ms=None):
        """HA failover: this rank now owns ``queues`` (Queue objects re-homed
        from a dead rank whose store is ``src``).  Their stored messages go into this
        plane — unacked ones first, flagged redelivered, then the ready ones in offset
        order — exactly like ``recover`` for a restart (reference: a re-homed QueueEntity
        reloads its rows from Cassandra, QueueEntity.scala:80-140).  The rows move into
        this rank's store (committed) before they are deleted from the dead rank's, so a
        crash in between duplicates rather than loses.  Returns messages restored."""
        p, st = self.plane, self.store
        if self.native is not None:
            self.native.drain()
        items, moved, seeds = [], [], []
        adopt_refs = {}
        for q in queues:
            if not q.durable:
                continue
            qid = entity_id(q.vhost, q.name)
            r = src.select_queue(qid)
            if r is None:   # declared through another rank: the dead rank stored only rows
                src.insert_queue_meta(qid, -1, set(), True, q.ttl_ms)
                r = src.select_queue(qid)
            (lconsumed, _, _, _), msgs, unacks = r
            order = [(off, mid, True) for off, mid, _ in sorted(unacks)] + \
                    [(off, mid, False) for off, mid, _ in sorted(msgs) if off > lconsumed]
            base = p.queue_tail(q.slot)
            st.insert_queue_meta(qid, -1, set(), True, q.ttl_ms)
            for i, (off, mid, red) in enumerate(order):
                m = src.select_message(mid)
                if m is None:
                    continue
                _, ts, header, body, ex, rk, _, _ = m
                items.append((q.slot, mid, ts, 0, ex.encode(), rk.encode(), header[10:], body, True, red))
                moved.append((qid, off, mid, red))
                # references of this message among the adopted rows (one message routed to
                # several of the dead rank's durable queues keeps one row with refer = n)
                refs = self.refs if self.native is None else adopt_refs
                n = refs.get(mid, 0)
                refs[mid] = n + 1
                if n == 0 and st.select_message(mid) is None:
                    st.insert_message(mid, ts, header, body, ex, rk, True, 1, 0)
                elif n:
                    st.update_message_refer_count(mid, n + 1)
                st.insert_queue_msg(qid, base + i, mid, len(body), 0)
                if self.native is None:
                    self.rows[(qid, mid)] = [base + i, len(body), False]
                else:
                    seeds.append((qid, mid, base + i, len(body)))
        n = p.restore(items, now_ms) if items else 0
        st.sync()
        for qid, mid, off, size in seeds:
            self.native.seed_row(qid, mid, off, size, False, adopt_refs[mid])
        # handed over: the dead rank's store no longer holds them (its restart must not
        # deliver them a second time)
        for qid, off, mid, red in moved:
            if red:
                src.delete_queue_unack(qid, mid)
            else:
                src.delete_queue_msg(qid, off)
            # a message row may still back another of the dead rank's queues that a
            # different survivor adopts (concurrently): drop only this queue's reference
            m = src.select_message(mid)
            if m is not None:
                if m[7] <= 1:
                    src.delete_message(mid)
                else:
                    src.update_message_refer_count(mid, m[7] - 1)
        for q in queues:
            if q.durable:
                src.force_delete_queue(entity_id(q.vhost, q.name))
        src.sync()
        return n

    # ------------------------------------------------------------------ recovery
    def recover(self, now_ms=0):
        """Durable topology + messages from the store into the plane.  Returns the number
        of messages restored."""
        p, st = self.plane, self.store
        for v in st.vhost_ids():
            p.ensure_vhost(v)
        binds = []
        for xid in st.exchange_ids():
            r = st.select_exchange(xid)
            if r is None:
                continue
            (tpe, durable, autodel, internal, args), bl = r
            v, name = _split_eid(xid)
            v = v or "AMQ.DEFAULT"
            p.ensure_vhost(v)
            p.declare_exchange(v, name, tpe, durable=durable, auto_delete=autodel, internal=internal,
                               arguments=args)
            binds += [(v, _split_eid(qid)[1], name, key) for qid, key, _ in bl]
        items, rewrite = [], []
        for qid in st.queue_ids():
            r = st.select_queue(qid)
            if r is None:
                continue
            (lconsumed, consumers, durable, ttl), msgs, unacks = r
            if not durable:
                continue
            v, name = _split_eid(qid)
            v = v or "AMQ.DEFAULT"
            p.ensure_vhost(v)
            slot = p.declare_queue(v, name, durable=True, ttl_ms=int(ttl or 0))
            order = [(off, mid, True) for off, mid, _ in sorted(unacks)] + \
                    [(off, mid, False) for off, mid, _ in sorted(msgs) if off > lconsumed]
            new_off = 0
            for off, mid, red in order:
                m = st.select_message(mid)
                if m is None:
                    continue
                _, ts, header, body, ex, rk, _, _ = m
                props = header[10:]
                items.append((slot, mid, ts, 0, ex.encode(), rk.encode(), props, body, True, red))
                rewrite.append((qid, off, new_off, mid, len(body), red))
                self.refs[mid] = self.refs.get(mid, 0) + 1
                new_off += 1
        for v, q, x, key in binds:
            if (v, q) in p.queues:
                p.bind(v, q, x, key)
        n = p.restore(items, now_ms) if items else 0
        # new ids strictly above every stored one (snowflake ms field), even if the device
        # clock ran ahead of the wall clock before the restart or the clock went back
        top = max((it[1] for it in items), default=0)
        for mid in st.message_ids() if hasattr(st, "message_ids") else ():
            top = max(top, mid)
        if top and hasattr(p, "seed_ids"):
            p.seed_ids((top >> 22) + 1)
        # device offsets restart at 0: move the rows to them
        for qid, off, new_off, mid, size, red in rewrite:
            if red:
                st.delete_queue_unack(qid, mid)
            else:
                st.delete_queue_msg(qid, off)
        for qid, off, new_off, mid, size, red in rewrite:
            st.insert_queue_msg(qid, new_off, mid, size, 0)
            st.insert_last_consumed(qid, -1)
            self.rows[(qid, mid)] = [new_off, size, False]
        st.sync()
        return n
