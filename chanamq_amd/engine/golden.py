"""Golden (pure Python) data plane with exactly the GPU step semantics.

Same ControlState API as GpuDataPlane; ``step()`` consumes the same ingress and
must produce byte-identical per-connection egress for deterministic scenarios
(one publishing connection per queue per step; no shared channel-level limits
across queues).  This is the executable specification of csrc/kernels/dataplane.hip
and the reference-semantics model the tests compare kernels against.
"""

import struct
from collections import defaultdict

import numpy as np

from ..models.matcher import topic_match
from ..protocol import constants as C
from .control import ControlState
from .layout import (MF_HAS_TS, MF_PERSIST, RDESC, SS_CTRL, SS_FRAME_ERROR, SS_OVERFLOW, SS_TOO_LARGE,
                     SS_UNEXPECTED)

NO_ROUTE_TEXT = C.REPLY_TEXT[312].encode()
NO_CONS_TEXT = C.REPLY_TEXT[313].encode()


def _frame(t, ch, payload):
    return struct.pack(">BHI", t, ch, len(payload)) + payload + b"\xce"


class _Msg:
    __slots__ = ("ex", "rk", "props", "body", "refcnt", "pub_step", "flags", "id", "ts", "restored")
    _next = 1

    def __init__(self, ex, rk, props, body, nq, step, flags, mid=None, ts=0):
        self.ex, self.rk, self.props, self.body = ex, rk, props, body
        self.refcnt, self.pub_step, self.flags = nq, step, flags
        if mid is None:
            mid, _Msg._next = _Msg._next, _Msg._next + 1
        self.id, self.ts, self.restored = mid, ts, False


class GoldenDataPlane(ControlState):
    def __init__(self, hash_wildcard=True, ucap=8192, deliver_cap=4096, carry_cap=1 << 20,
                 egress_cap=96 << 20, deliv_max=65536, exchanger=None, xfer_desc_max=1 << 15,
                 xfer_bytes=1 << 24, persist=False, exchange_lag=0, persist_max=1 << 16, deliver_cap_bytes=0, **kw):
        super().__init__(hash_wildcard=hash_wildcard, **kw)
        self.persist = persist
        # k_dequeue: durable TTL skips <= persist_max / 4 a step; the engine raises
        # persist_max to 2 * deliv_max + 4096 (a step's consumed records always fit)
        self.persist_max = max(persist_max, 2 * deliv_max + 4096) if persist else persist_max
        self._ttl_budget = 0
        self.lag = bool(exchange_lag) and self.world > 1
        self._lag_prev = []                 # exchange_lag: records received last step
        self._persist_out, self._consumed_out = [], []
        self.link_slots = set()   # shadow queues of remote consumers: consumed records always
        self.exchanger = exchanger
        self._outbox = defaultdict(list)  # dest rank -> [(RDesc fields, payload)]
        self._deferred = []                # this rank's routed publishes awaiting step_b
        self._pend = None
        if self.world > 1:
            import torch
            self._xs_desc = torch.zeros(xfer_desc_max * RDESC.itemsize, dtype=torch.uint8)
            self._xs_pay = torch.zeros(xfer_bytes, dtype=torch.uint8)
            self._xr_desc = torch.zeros(xfer_desc_max * RDESC.itemsize, dtype=torch.uint8)
            self._xr_pay = torch.zeros(xfer_bytes, dtype=torch.uint8)
        self.ucap, self.deliver_cap, self.carry_cap = ucap, deliver_cap, carry_cap
        self.deliver_cap_bytes = int(deliver_cap_bytes)
        self.egress_cap, self.deliv_max = egress_cap, deliv_max
        self.carry = defaultdict(bytes)
        self.step_no = 0
        self.ring = defaultdict(list)     # queue slot -> [(msg, redelivered, expire)]
        self.qrr = defaultdict(int)
        self.ch = {}                      # chslot -> dict state
        self.cons_unacked = defaultdict(int)
        self.dirty = []
        self.requeue_items = []           # (q, msg, qpos, expire)
        self.qpos_head = defaultdict(int)  # absolute position of ring[0]
        self.counters = defaultdict(int)

    # ------------------------------------------------------------------ hooks
    def channel_opened(self, chan):
        s = chan.conn * self.chpc + chan.local
        self.ch[s] = dict(next_tag=1, uhead=1, ack_upto=0, req_upto=0, confirm_next=1, pub_cnt=0,
                          unacked=0, win=0, slots={}, dirty=False, num=chan.ch)

    def channel_closing(self, chan):
        s = chan.conn * self.chpc + chan.local
        self.ch[s]["req_upto"] = 1 << 62
        self._mark_dirty(s)

    def queue_declared(self, q):
        self.ring[q.slot] = []
        self.qpos_head[q.slot] = 0
        self.qrr[q.slot] = 0

    # ---- persistence (same records as the GPU plane's take_persist / take_consumed)
    def _consumed(self, msg, q, qpos, kind):
        qq = self.queue_by_slot.get(q)
        if (self.persist or q in self.link_slots) and qq is not None and qq.durable and (msg.flags & MF_PERSIST):
            self._consumed_out.append((msg.id, q, qpos, kind))

    def take_link_consumed(self, slots):
        """Consumed records of the remote-consumer shadow queues ``slots`` (parallel/
        links.py), taken out; the rest stay for the persistence layer."""
        mine = [r for r in self._consumed_out if r[1] in slots]
        if mine:
            self._consumed_out = [r for r in self._consumed_out if r[1] not in slots]
        return mine

    def _mid(self):
        """Message ids unique across ranks (the device uses per-GPU snowflake workers):
        a rank's store may be adopted by a survivor whose own ids must not collide."""
        _Msg._next += 1
        return _Msg._next * 1024 + self.rank if self.world > 1 else _Msg._next

    def queue_tail(self, q):
        """Queue position the next enqueue into slot ``q`` gets."""
        return self.qpos_head[q] + len(self.ring[q])

    def take_persist(self):
        out, self._persist_out = self._persist_out, []
        return out

    def take_consumed(self):
        out, self._consumed_out = self._consumed_out, []
        return out

    def restore(self, items, now_ms=0):
        n = 0
        for q, mid, ts, exp, ex, rk, props, body, persistent, red in items:
            qq = self.queue_by_slot[q]
            ring = self.ring[q]
            if len(ring) >= qq.capacity:
                continue
            msg = _Msg(ex, rk, props, body, 1, self.step_no, MF_PERSIST if persistent else 0, mid=mid, ts=ts)
            msg.restored = True
            ring.append((msg, bool(red), exp))
            n += 1
        return n

    def memory_in_use(self):
        seen, tot = set(), 0
        for ring in self.ring.values():
            for m, _, _ in ring:
                if id(m) not in seen:
                    seen.add(id(m))
                    tot += len(m.ex) + len(m.rk) + len(m.props) + len(m.body)
        return tot

    def message_count(self, q):
        return len(self.ring[q])

    def purge(self, q):
        ring = self.ring[q]
        self.ring[q] = [(m, red, 1) for (m, red, _) in ring]   # released by the next dequeue
        return len(ring)

    def recover(self, conn, ch):
        s = self.chslot(conn, ch)
        st = self.ch[s]
        st["req_upto"] = max(st["req_upto"], st["next_tag"] - 1)
        self._mark_dirty(s)

    def unpause(self, conn):
        c = self.conns.get(conn)
        if c is not None:
            c.paused = False

    def _ack_mark(self, s, tag, multiple, requeue):
        st = self.ch[s]
        if tag == 0 and multiple:
            tag = st["next_tag"] - 1
        if multiple:   # resolved in wire order at the window advance: first cover wins
            st.setdefault("msettles", []).append((tag, bool(requeue)))
        elif st["uhead"] <= tag < st["next_tag"]:
            sl = st["slots"].get(tag)
            if sl and sl["state"] == "pending":
                sl["state"] = "requeue" if requeue else "acked"
        self._mark_dirty(s)

    def apply_ack(self, conn, ch, tag, multiple=False, requeue=False, kind="ack"):
        """Ack / Nack / Reject between steps (Tx.Commit), like GpuDataPlane.apply_ack."""
        self._ack_mark(self.chslot(conn, ch), tag, multiple, bool(requeue) and kind != "ack")

    def basic_get(self, conn, ch, q, no_ack, now_ms=0):
        """Basic.Get between steps: spec of k_basic_get (dataplane.hip)."""
        ring = self.ring[q]
        while ring and ring[0][2] and ring[0][2] <= now_ms:
            self._consumed(ring[0][0], q, self.qpos_head[q], 1)
            self._release(ring.pop(0)[0])
            self.qpos_head[q] += 1
        if not ring:
            return None, 0
        s = self.chslot(conn, ch)
        st = self.ch[s]
        if st["win"] >= self.ucap:
            from .control import ControlError
            raise ControlError(C.RESOURCE_ERROR, "basic.get: channel delivery window full", 60, 70)
        msg, red, exp = ring.pop(0)
        qpos = self.qpos_head[q]
        self.qpos_head[q] += 1
        tag = st["next_tag"]
        st["next_tag"] += 1
        st["win"] += 1
        st["slots"][tag] = dict(state="done" if no_ack else "pending", msg=msg, q=q, cons=-1, qpos=qpos, expire=exp)
        if no_ack:
            self._consumed(msg, q, qpos, 0)
            self._release(msg)
        else:
            st["unacked"] += 1
            self.cons_unacked[-1] += 1
            self._consumed(msg, q, qpos, 3)
        self._mark_dirty(s)
        fm = self.conns[conn].frame_max
        mp = (struct.pack(">HHQB", 60, 71, tag, 1 if red else 0) + bytes([len(msg.ex)]) + msg.ex
              + bytes([len(msg.rk)]) + msg.rk + struct.pack(">I", len(ring)))
        parts = [_frame(1, st["num"], mp), _frame(2, st["num"], struct.pack(">HHQ", 60, 0, len(msg.body)) + msg.props)]
        step = fm - 8 if fm else len(msg.body)
        for i in range(0, len(msg.body), max(step, 1)):
            parts.append(_frame(3, st["num"], msg.body[i:i + step]))
        return b"".join(parts), len(ring)

    def _mark_dirty(self, s):
        if not self.ch[s]["dirty"]:
            self.ch[s]["dirty"] = True
            self.dirty.append(s)

    def _chan_of(self, conn, ch):
        c = self.conns.get(conn)
        if c is None or ch == 0 or ch not in c.channels:
            return None
        return conn * self.chpc + c.channels[ch].local

    def _dget_resolve(self, conn, data, p, size):
        """Basic.Get the step serves itself (spec of dget_resolve, dataplane.hip): a named
        queue bound to the vhost's default exchange, owned here, not another connection's
        exclusive queue.  -> (queue slot, no_ack) or None (the host serves it)."""
        if size < 8:
            return None
        a, end = p + 7 + 6, p + 7 + size
        n = data[a]
        if n == 0 or a + 1 + n + 1 > end:
            return None
        name = bytes(data[a + 1:a + 1 + n])
        x = self.exchanges.get((self.conns[conn].vhost, ""))
        if x is None or x.type != "direct":
            return None
        qs = self._route(x, name)
        if len(qs) != 1:
            return None
        q = self.queue_by_slot.get(qs[0])
        if q is None or q.owner != self.rank or q.exclusive_owner not in (-1, conn):
            return None
        return q.slot, data[a + 1 + n] & 1

    # ------------------------------------------------------------------ frame scan (K1)
    def _scan(self, conn, data):
        c = self.conns[conn]
        fmax = c.frame_max
        L = len(data)
        frames = []
        pos = 0
        err = None
        while pos < L:
            if L - pos < 7:
                frames.append((pos, None))
                break
            t, ch, size = struct.unpack_from(">BHI", data, pos)
            if t not in (1, 2, 3, 8) or (fmax and size + 8 > fmax):
                err = 3
                break
            if pos + 8 + size > L:
                frames.append((pos, None))
                break
            if data[pos + 7 + size] != 0xCE:
                err = 3
                break
            frames.append((pos, (t, ch, size)))
            pos += 8 + size
        end_pos = pos
        cmds = []
        stop = None  # (frame index, reason)
        f = 0
        nf = len(frames)
        gkey = None   # (channel, queue, no_ack) of the segment's first step-served Basic.Get
        while f < nf:
            p, fi = frames[f]
            if fi is None:
                stop = (f, 1)
                break
            t, ch, size = fi
            if t == 8:
                f += 1
                continue
            if t != 1:
                stop = (f, 2)
                break
            if size < 4:
                stop = (f, 3)
                break
            cls, mid = struct.unpack_from(">HH", data, p + 7)
            chs = self._chan_of(conn, ch)
            g = self._dget_resolve(conn, data, p, size) if (cls, mid) == (60, 70) and chs is not None else None
            if gkey is not None and (g is None or (ch,) + g != gkey):
                stop = (f, 4)   # only the same Basic.Get may follow the first in one step
                break
            if g is not None:
                gkey = (ch,) + g
                cmds.append(dict(kind="get", ch=ch, chslot=chs, q=g[0], noack=bool(g[1]), raw=data[p:p + 8 + size]))
                f += 1
                continue
            data_cmd = cls == 60 and mid in (40, 80, 90, 120) and chs is not None
            if cls == 60 and mid == 40:
                if f + 1 >= nf or frames[f + 1][1] is None:
                    stop = (f, 1)
                    break
                hp, hi = frames[f + 1]
                if hi[0] != 2 or hi[1] != ch or hi[2] < 14:
                    stop = (f, 2)
                    break
                bsz = struct.unpack_from(">Q", data, hp + 7 + 4)[0]
                got, e, bad, inc = 0, f + 1, None, False
                bodies = []
                while got < bsz:
                    e += 1
                    if e >= nf or frames[e][1] is None:
                        inc = True
                        break
                    bp, bi = frames[e]
                    if bi[0] != 3 or bi[1] != ch:
                        bad = 2
                        break
                    got += bi[2]
                    bodies.append((bp + 7, bi[2]))
                    if got > bsz:
                        bad = 3
                        break
                if inc:
                    stop = (f, 1)
                    break
                if bad:
                    stop = (f, bad)
                    break
                endp = (frames[e][0] + 8 + frames[e][1][2])
                cmd = dict(kind="publish" if data_cmd else "control", ch=ch, chslot=chs,
                           m=(p + 7, size), h=(hp + 7, hi[2]), bodies=bodies, bsz=bsz,
                           raw=data[p:endp])
                cmds.append(cmd)
                f = e + 1
                if not data_cmd:
                    stop = (f, 0)
                    break
                continue
            endp = p + 8 + size
            kind = {80: "ack", 90: "reject", 120: "nack"}.get(mid) if (cls == 60 and data_cmd) else "control"
            cmds.append(dict(kind=kind, ch=ch, chslot=chs, m=(p + 7, size), raw=data[p:endp]))
            f += 1
            if kind == "control":
                stop = (f, 0)
                break
        if stop is None:
            if err is not None:
                stop = (nf, 3)
            else:
                stop = (nf, 7)
        kf, reason = stop
        consumed = frames[kf][0] if kf < nf else (end_pos if err is None or True else end_pos)
        if kf >= nf:
            consumed = end_pos
        status = 0
        if reason in (2, 3):
            status |= SS_FRAME_ERROR if reason == 3 else SS_UNEXPECTED
        if reason == 0:
            status |= SS_CTRL
        if reason == 4:
            status |= SS_OVERFLOW
        return cmds, consumed, status

    # ------------------------------------------------------------------ one step
    def step(self, inputs=None, now_ms=0):
        """One step.  Sharded (world > 1): phase A, the all-to-all through ``exchanger``,
        phase B — ``LocalCluster`` drives the phases itself for in-process clusters."""
        self.step_a(inputs, now_ms)
        if self.world > 1:
            if self.exchanger is None:
                raise RuntimeError("sharded golden plane needs an exchanger (or a LocalCluster)")
            recv = self.exchanger.exchange(self.pending_send_counts(), self._xs_desc, self._xs_pay,
                                           self._xr_desc, self._xr_pay)
            return self.step_b(recv)
        return self.step_b(None)

    # exchange operands (parallel/exchange.py)
    def xfer_send_desc(self):
        return self._xs_desc

    def xfer_send_pay(self):
        return self._xs_pay

    def xfer_recv_desc(self):
        return self._xr_desc

    def xfer_recv_pay(self):
        return self._xr_pay

    def pending_send_counts(self):
        return self._pend["send_counts"]

    def _pack(self):
        """Serialise the outbox destination-major (same layout as k_pack)."""
        W = self.world
        n, b = [0] * W, [0] * W
        recs = []
        for r in range(W):
            for fields, payload in self._outbox.get(r, []):
                recs.append((r, fields, payload))
        desc = np.zeros(len(recs), RDESC)
        pay = bytearray()
        for r in range(W):
            rel = 0
            for fields, payload in self._outbox.get(r, []):
                k = sum(n)
                f = dict(fields)
                f["pay_off"] = rel
                for key, v in f.items():
                    desc[k][key] = v
                padded = payload + b"\0" * ((-len(payload)) % 16)
                pay += padded
                rel += len(padded)
                n[r] += 1
                b[r] += len(padded)
        self._outbox = defaultdict(list)
        if desc.nbytes > self._xs_desc.numel() or len(pay) > self._xs_pay.numel():
            raise RuntimeError("golden exchange buffers too small")
        import torch
        if len(desc):
            self._xs_desc[:desc.nbytes] = torch.from_numpy(desc.view(np.uint8).copy())
        if pay:
            self._xs_pay[:len(pay)] = torch.frombuffer(bytearray(pay), dtype=torch.uint8)
        return n + b

    def _parse_recv(self, recv):
        """Received records -> [(source rank, exch, flags, expire, ex, rk, props, body)]."""
        W = self.world
        rn, rb = recv[:W], recv[W:2 * W]
        tot = sum(rn)
        if not tot:
            return []
        desc = self._xr_desc[:tot * RDESC.itemsize].numpy().view(RDESC)
        pay = self._xr_pay[:sum(rb)].numpy().tobytes()
        pbase = [sum(rb[:s]) for s in range(W)]
        out, i = [], 0
        for s in range(W):
            for _ in range(rn[s]):
                d = desc[i]
                i += 1
                o = pbase[s] + int(d["pay_off"])
                exl, rkl, pl, bl = int(d["ex_len"]), int(d["rk_len"]), int(d["props_len"]), int(d["body_len"])
                out.append((s, int(d["exch"]), int(d["flags"]), int(d["expire_ms"]), pay[o:o + exl],
                            pay[o + exl:o + exl + rkl], pay[o + exl + rkl:o + exl + rkl + pl],
                            pay[o + exl + rkl + pl:o + exl + rkl + pl + bl]))
        return out

    def _import(self, records, now_ms):
        """Enqueue the step's messages in (source rank, connection, publish) order: this
        rank's own publishes at its rank position, records from rank s at s's — the
        order the GPU pair sort produces with its (queue, source rank) keys."""
        by_src = defaultdict(list)
        for r in records:
            by_src[r[0]].append(r)
        for s in range(self.world):
            if s == self.rank:
                for msg, qs, expire, chslot in self._deferred:
                    self._enqueue(msg, qs, expire, now_ms, chslot)
                self._deferred = []
            for _, exch, flags, expire, ex, rk, props, body in by_src.get(s, []):
                x = self.exch_by_slot.get(exch)
                if x is None:
                    continue
                qs = [q for q in self._route(x, rk) if self.queue_by_slot[q].owner == self.rank]
                if not qs:
                    continue
                msg = _Msg(ex, rk, props, body, len(qs), self.step_no, flags & MF_PERSIST, mid=self._mid())
                self._enqueue(msg, qs, expire, now_ms)

    def step_a(self, inputs=None, now_ms=0):
        inputs = inputs or {}
        self.counters = defaultdict(int)
        cnt = self.counters
        out = {"egress": {}, "ctrl": [], "txbuf": [], "events": [], "segs": []}
        conns = {c for c in inputs if c in self.conns}   # bytes of a connection closed meanwhile: dropped
        for c, cl in self.carry.items():
            if cl and c in self.conns and not self.conns[c].paused:
                conns.add(c)
        pubs, acks, gets = [], [], []
        for conn in sorted(conns):
            data = self.carry[conn] + inputs.get(conn, b"")
            if self.conns[conn].paused:
                self.carry[conn] = data
                out["segs"].append((conn, 1, 0, len(data)))
                continue
            cmds, consumed, status = self._scan(conn, data)
            chans = self.conns[conn].channels
            for cmd in cmds:
                cmd["conn"] = conn
                if cmd["kind"] == "get":
                    gets.append(cmd)
                elif cmd["kind"] != "control" and chans[cmd["ch"]].tx:   # held until Tx.Commit
                    out["txbuf"].append((conn, cmd["m"][0] - 7, cmd["raw"]))
                elif cmd["kind"] == "publish":
                    pubs.append((cmd, data))
                elif cmd["kind"] in ("ack", "reject", "nack"):
                    acks.append((cmd, data))
                else:
                    out["ctrl"].append((conn, cmd["raw"]))
            rest = data[consumed:]
            if len(rest) > self.carry_cap:
                status |= SS_TOO_LARGE
                rest = b""
            self.carry[conn] = rest
            if status & SS_CTRL:
                self.conns[conn].paused = True
            out["segs"].append((conn, status, consumed, len(rest)))
        # ---- publishes: decode, route, returns, store, enqueue
        returns = defaultdict(list)
        for cmd, data in pubs:
            self._publish(cmd, data, now_ms, returns, out)
        self._pend = dict(out=out, returns=returns, acks=acks, gets=gets, now_ms=now_ms,
                          send_counts=self._pack() if self.world > 1 else None)

    def step_b(self, recv=None):
        st, self._pend = self._pend, None
        out, returns, acks, now_ms = st["out"], st["returns"], st["acks"], st["now_ms"]
        dgets = st.get("gets", ())
        cnt = self.counters
        if recv is not None:
            records = self._parse_recv(recv)
            if self.lag:   # exchange_lag: import what arrived last step, keep this step's
                records, self._lag_prev = self._lag_prev, records
            self._import(records, now_ms)
        # ---- acks
        for cmd, data in acks:
            o = cmd["m"][0] + 4
            tag = struct.unpack_from(">Q", data, o)[0]
            bits = data[o + 8]
            kind = cmd["kind"]
            multiple = bool(bits & 1) if kind != "reject" else False
            requeue = (bits & 1) if kind == "reject" else ((bits >> 1) & 1 if kind == "nack" else 0)
            self._ack_mark(cmd["chslot"], tag, multiple, requeue)
            cnt["n_acked"] += 1
        # ---- window advance (k_chan_advance)
        dirty, self.dirty = self.dirty, []
        for s in dirty:
            st = self.ch[s]
            st["dirty"] = False
            contiguous = True
            t = st["uhead"]
            released = 0
            # multiple settles of the step: record-breaking uptos in wire order (a tag's
            # fate is the first settle that covers it; spec of chan_advance_one)
            marks, top = [], 0
            for up, rq in st.pop("msettles", ()):
                if up > top:
                    marks.append((up, rq))
                    top = up
            while t < st["next_tag"]:
                sl = st["slots"].get(t)
                state = sl["state"]
                if state == "pending":
                    if t <= st["ack_upto"]:
                        state = "acked"
                    elif t <= st["req_upto"]:
                        state = "requeue"
                    else:
                        for up, rq in marks:
                            if t <= up:
                                state = "requeue" if rq else "acked"
                                break
                if state == "acked":
                    self._consumed(sl["msg"], sl["q"], sl["qpos"], 0)
                    self._release(sl["msg"])
                    self.cons_unacked[sl["cons"]] -= 1
                    st["unacked"] -= 1
                    state = "done"
                elif state == "requeue":
                    self._consumed(sl["msg"], sl["q"], sl["qpos"], 4)
                    self.requeue_items.append((sl["q"], sl["msg"], sl["qpos"], sl["expire"]))
                    self.cons_unacked[sl["cons"]] -= 1
                    st["unacked"] -= 1
                    cnt["n_requeue"] += 1
                    state = "done"
                sl["state"] = state
                if contiguous and state == "done":
                    released += 1
                else:
                    contiguous = False
                t += 1
            for k in range(st["uhead"], st["uhead"] + released):
                st["slots"].pop(k, None)
            st["uhead"] += released
            st["win"] -= released
        # requeue (k_requeue): back in front of the heads, per queue in queue-position order,
        # before this step's dispatch
        if self.requeue_items:
            byq = defaultdict(list)
            for it in self.requeue_items:
                byq[it[0]].append(it)
            self.requeue_items = []
            for q, items in byq.items():
                items.sort(key=lambda x: x[2])
                ring = self.ring[q]
                cap = self.queue_by_slot[q].capacity if q in self.queue_by_slot else 0
                free = cap - len(ring)
                k = min(len(items), free)
                self.ring[q] = [(m, True, e) for (_, m, _, e) in items[:k]] + ring
                self.qpos_head[q] -= k
                self.requeue_items.extend(items[k:])
        # ---- dequeue (k_dequeue)
        delivs = []
        budget = [0]
        self._ttl_budget = 0
        gets = defaultdict(list)
        for g in dgets:
            gets[g["q"]].append(g)
        gempty = defaultdict(list)
        for q in sorted(self.queue_by_slot):
            delivs.extend(self._dequeue(q, now_ms, budget, gets.get(q, ()), gempty, out))
        # ---- tags: stable sort by chslot
        delivs.sort(key=lambda d: d["chslot"])
        for d in delivs:
            st = self.ch[d["chslot"]]
            d["tag"] = st["next_tag"]
            st["next_tag"] += 1
            st["slots"][d["tag"]] = dict(state="done" if d["noack"] else "pending", msg=d["msg"],
                                         q=d["q"], cons=d["cons"], qpos=d["qpos"], expire=d["expire"])
            if not d["noack"]:
                self._consumed(d["msg"], d["q"], d["qpos"], 3)
            self._mark_dirty(d["chslot"])
            cnt["lat_" + str(min(self.step_no - d["msg"].pub_step, 31))] += 1
        # ---- egress per connection: returns, confirms, deliveries
        by_conn = defaultdict(list)
        for d in delivs:
            by_conn[d["chslot"] // self.chpc].append(d)
        conns_out = set(by_conn) | set(returns) | set(gempty)
        for s, st in self.ch.items():
            if st["pub_cnt"]:
                conns_out.add(s // self.chpc)
        for conn in sorted(conns_out):
            parts = list(returns.get(conn, []))
            for local in range(self.chpc):
                s = conn * self.chpc + local
                st = self.ch.get(s)
                if not st or not st["pub_cnt"]:
                    continue
                n = st["pub_cnt"]
                st["pub_cnt"] = 0
                last = st["confirm_next"] + n - 1
                st["confirm_next"] = last + 1
                mid = 120 if st.pop("pub_fail", False) else 80
                parts.append(_frame(1, st["num"], struct.pack(">HHQB", 60, mid, last, 1 if n > 1 else 0)))
            fm = self.conns[conn].frame_max if conn in self.conns else 131072
            for d in by_conn.get(conn, []):
                parts.append(self._render_deliver(d, fm))
            for chno in gempty.get(conn, ()):   # Basic.GetEmpty frames close the region
                parts.append(_frame(1, chno, struct.pack(">HHB", 60, 72, 0)))
            if parts:
                out["egress"][conn] = b"".join(parts)
        for d in delivs:
            if d["noack"]:
                self._consumed(d["msg"], d["q"], d["qpos"], 0)
                self._release(d["msg"])
        cnt["n_deliv"] = len(delivs)
        self.step_no += 1
        out["counters"] = dict(cnt)
        return out

    def _release(self, msg):
        msg.refcnt -= 1
        if msg.refcnt == 0:
            self.counters["n_freed"] += 1

    def _publish(self, cmd, data, now_ms, returns, out):
        conn = cmd["conn"]
        cnt = self.counters
        mo, ml = cmd["m"]
        o = mo + 6
        exl = data[o]
        ex = data[o + 1:o + 1 + exl]
        o += 1 + exl
        rkl = data[o]
        rk = data[o + 1:o + 1 + rkl]
        o += 1 + rkl
        bits = data[o]
        mandatory, immediate = bool(bits & 1), bool(bits & 2)
        ho, hl = cmd["h"]
        props = data[ho + 12:ho + hl]
        body = b"".join(data[bo:bo + bl] for bo, bl in cmd["bodies"])
        s = cmd["chslot"]
        st = self.ch[s]
        chan = self.conns[conn].channels[cmd["ch"]]
        if chan.confirm:
            st["pub_cnt"] += 1
        expire = self._expiration(props, now_ms)
        vhost = self.conns[conn].vhost
        x = self.exchanges.get((vhost, ex.decode("utf-8", "surrogateescape")))
        if x is None:
            cnt["n_unknown_exchange"] += 1
            out["events"].append((conn, 404, s))
            return
        qs = self._route(x, rk)
        remote = sorted({self.queue_by_slot[q].owner for q in qs} - {self.rank}) if self.world > 1 else []
        ret = 0
        if not qs:
            cnt["n_unroutable"] += 1
            if mandatory:
                ret = 312
        elif immediate and not remote and not any(self.queue_by_slot[q].consumers for q in qs):
            ret = 313
            qs = []
        if remote and not ret:
            fl = (MF_PERSIST if self._persistent(props) else 0)
            if self._prop_fields(props).get("timestamp") is not None:
                fl |= MF_HAS_TS
            fields = dict(body_len=len(body), props_len=len(props), exch=x.slot, flags=fl, ex_len=len(ex),
                          rk_len=len(rk), expire_ms=expire, ts_ms=0)
            for r in remote:
                self._outbox[r].append((fields, ex + rk + props + body))
            qs = [q for q in qs if self.queue_by_slot[q].owner == self.rank]
        if ret:
            txt = NO_ROUTE_TEXT if ret == 312 else NO_CONS_TEXT
            fm = self.conns[conn].frame_max
            mp = struct.pack(">HHHB", 60, 50, ret, len(txt)) + txt + bytes([len(ex)]) + ex + bytes([len(rk)]) + rk
            fr = [_frame(1, cmd["ch"], mp), _frame(2, cmd["ch"], struct.pack(">HHQ", 60, 0, len(body)) + props)]
            step = fm - 8 if fm else len(body)
            for i in range(0, len(body), max(step, 1)):
                fr.append(_frame(3, cmd["ch"], body[i:i + step]))
            returns[conn].append(b"".join(fr))
        if not qs:
            return
        flags = 1 if self._persistent(props) else 0
        tsp = self._prop_fields(props).get("timestamp")
        msg = _Msg(ex, rk, props, body, len(qs), self.step_no, flags, ts=int(tsp) * 1000 if tsp else 0,
                   mid=self._mid())
        if self.world > 1:   # enqueued in step_b, ordered by source rank (see _import)
            self._deferred.append((msg, qs, expire, s))
        else:
            self._enqueue(msg, qs, expire, now_ms, s)

    def _enqueue(self, msg, qs, expire, now_ms, chslot=None):
        cnt = self.counters
        for q in qs:
            qq = self.queue_by_slot[q]
            ring = self.ring[q]
            if len(ring) >= qq.capacity:   # the device grows the ring before enqueueing (k_ring_plan)
                new = self.grow_target(qq, len(ring) + 1)
                if new is not None:
                    self.regrow_ring(qq, new)
            if len(ring) >= qq.capacity:
                cnt["n_ring_full"] += 1
                self._release(msg)
                if chslot is not None:   # the publisher gets Basic.Nack for this step's range
                    self.ch[chslot]["pub_fail"] = True
                continue
            e = expire
            if qq.ttl_ms > 0:
                qe = now_ms + qq.ttl_ms
                e = qe if (e == 0 or qe < e) else e
            if self.persist and qq.durable and (msg.flags & MF_PERSIST) and not msg.restored:
                self._persist_out.append((msg.id, msg.ts, q, self.qpos_head[q] + len(ring), e, msg.ex, msg.rk,
                                          msg.props, msg.body))
            ring.append((msg, False, e))

    def _route(self, x, rk):
        if x.type == "direct":
            seen = []
            for q, k in x.bindings:
                if k == rk and q not in seen:
                    seen.append(q)
            return sorted(seen)
        if x.type == "fanout":
            return sorted({q for q, _ in x.bindings})
        out = []
        key = rk.decode("utf-8", "surrogateescape")
        for q, k in sorted(set(x.bindings)):
            if out and out[-1] == q:
                continue
            if topic_match(k.decode("utf-8", "surrogateescape"), key, self.hash_wildcard):
                out.append(q)
        return out

    @staticmethod
    def _prop_fields(props):
        from ..protocol.codec import decode_properties
        try:
            p, _ = decode_properties(props)
        except Exception:
            return {}
        return p

    def _persistent(self, props):
        return self._prop_fields(props).get("delivery_mode") == 2

    def _expiration(self, props, now_ms):
        e = self._prop_fields(props).get("expiration")
        if e and e.isdigit() and len(e) <= 18:
            return now_ms + int(e)
        return 0

    def _dequeue(self, q, now_ms, budget, gets=(), gempty=None, step_out=None):
        qq = self.queue_by_slot[q]
        ring = self.ring[q]
        cnt = self.counters
        budget_q = self.persist and qq.durable
        left = 0
        while ring and ring[0][2] and ring[0][2] <= now_ms:
            if budget_q and not left:   # reserved 64 at a time (dataplane.hip k_dequeue)
                if self._ttl_budget + 64 > self.persist_max >> 2:
                    break
                self._ttl_budget += 64
                left = 64
            left -= 1
            self._consumed(ring[0][0], q, self.qpos_head[q], 1)
            self._release(ring.pop(0)[0])
            self.qpos_head[q] += 1
            cnt["n_expired"] += 1
        # the step's Basic.Gets of this queue, in wire order, ahead of its consumers (spec of
        # k_dequeue's request loop): GetOk as a delivery on the getter's channel, GetEmpty at
        # the end of its connection's egress, a full delivery window -> the host serves it
        got = []
        for g in gets:
            s = g["chslot"]
            st = self.ch[s]
            if not ring:
                gempty[g["conn"]].append(st["num"])
                continue
            if st["win"] >= self.ucap or len(got) >= 32:   # (RUNS_PER_Q / 2 Get runs per queue)
                step_out["ctrl"].append((g["conn"], g["raw"], True))
                continue
            msg, red, exp = ring.pop(0)
            st["win"] += 1
            if not g["noack"]:
                st["unacked"] += 1
                self.cons_unacked[-1] += 1
            got.append(dict(chslot=s, cons=-1, msg=msg, q=q, qpos=self.qpos_head[q], expire=exp, redelivered=red,
                            noack=g["noack"], get_left=len(ring)))
            self.qpos_head[q] += 1
        mall = len(qq.consumers)
        if not mall or not ring:
            return got
        m = min(mall, 64 - len(got))
        r = self.qrr[q] % mall
        remaining = n_ring = len(ring)
        grants = []
        for j in range(m):
            cid = qq.consumers[(r + j) % mall]
            c = self.consumers[cid]
            chan = self.conns[c.conn].channels[c.ch]
            s = self.chslot(c.conn, c.ch)
            st = self.ch[s]
            g = 0
            if remaining and c.active and chan.flow:
                share = -(-remaining // (m - j))
                want = min(share, self.deliver_cap)
                cap = self.deliver_cap_bytes
                if cap and want > 1:   # byte cap: max(1, cap / size of the consumer's first delivery)
                    s0 = self._deliver_size(c, ring[n_ring - remaining][0])
                    want = min(want, 1 if s0 >= cap else cap // s0)
                pc = chan.prefetch_count
                if not c.no_ack and pc and not chan.global_:
                    want = min(want, max(pc - self.cons_unacked[cid], 0))
                g = min(want, self.ucap - st["win"])
                st["win"] += g
                if not c.no_ack and pc and chan.global_ and g:
                    g2 = min(g, max(pc - st["unacked"], 0))
                    st["win"] -= g - g2
                    st["unacked"] += g2
                    g = g2
                elif not c.no_ack and g:
                    st["unacked"] += g
                if not c.no_ack and g:
                    self.cons_unacked[cid] += g
            grants.append([cid, g])
            remaining -= g
        out = []
        pos = 0
        for cid, g in grants:
            if not g:
                continue
            c = self.consumers[cid]
            chan_s = self.chslot(c.conn, c.ch)
            for k in range(g):
                msg, red, exp = ring[pos + k]
                out.append(dict(chslot=chan_s, cons=cid, msg=msg, q=q, qpos=self.qpos_head[q] + pos + k,
                                expire=exp, redelivered=red, noack=c.no_ack, tag_str=c.tag.encode()))
            pos += g
        self.qrr[q] = (r + 1) % mall
        del ring[:pos]
        self.qpos_head[q] += pos
        return got + out

    def set_deliver_cap_bytes(self, n):
        self.deliver_cap_bytes = int(n)

    def _deliver_size(self, c, m):
        """Rendered size of a Basic.Deliver of m to consumer c (k_dequeue's deliver_size)."""
        fm = self.conns[c.conn].frame_max
        mp = 4 + 1 + len(c.tag.encode()[:255]) + 8 + 1 + 1 + len(m.ex) + 1 + len(m.rk)
        fmb = fm - 8 if fm else None
        nb = (-(-len(m.body) // fmb) if fmb else 1) if m.body else 0
        return 8 + mp + 8 + 12 + len(m.props) + len(m.body) + 8 * nb

    def _render_deliver(self, d, fm):
        m = d["msg"]
        ch = self.ch[d["chslot"]]["num"]
        if "get_left" in d:   # Basic.GetOk (message-count: what the queue held after it)
            mp = (struct.pack(">HHQB", 60, 71, d["tag"], 1 if d["redelivered"] else 0) + bytes([len(m.ex)]) + m.ex
                  + bytes([len(m.rk)]) + m.rk + struct.pack(">I", d["get_left"]))
        else:
            tag = d["tag_str"][:255]
            mp = (struct.pack(">HHB", 60, 60, len(tag)) + tag + struct.pack(">QB", d["tag"], 1 if d["redelivered"] else 0)
                  + bytes([len(m.ex)]) + m.ex + bytes([len(m.rk)]) + m.rk)
        parts = [_frame(1, ch, mp), _frame(2, ch, struct.pack(">HHQ", 60, 0, len(m.body)) + m.props)]
        step = fm - 8 if fm else len(m.body)
        for i in range(0, len(m.body), max(step, 1)):
            parts.append(_frame(3, ch, m.body[i:i + step]))
        return b"".join(parts)
