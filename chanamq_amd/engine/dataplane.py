"""GPU data plane: host control tables -> device tables, and the per-step driver.

``GpuDataPlane`` owns one ``_dataplane.Engine`` (HIP, gfx950).  Control-plane ops
(declare/bind/consume/qos/...) mutate ``ControlState`` and push the affected device
tables between steps; ``step()`` hands the step's ingress bytes to the captured
hipGraph and returns per-connection egress bytes plus the control commands the
device routed back to the host.
"""

import ctypes
import time
from collections import defaultdict

import os

import numpy as np

from .. import ops
from ..protocol import constants as C
from .control import ControlError, ControlState
from .layout import (CONN_OUT, CONSUMED_REC, EGRESS_REF, RING_MOVE, CTRL_REC, CTRL_DGET, CTRL_TXBUF, INVALID, MF_HAS_TS,
                     MF_HOSTPUB, MF_PERSIST,
                     MF_ONEQ, MF_REDELIVERED, MF_RESTORE,
                     PERSIST_HDR, RDESC, SEG_IN, SEG_OUT, SS_CTRL, US_ACKED, US_PENDING, US_REQUEUE, USLOT,
                     chan_hash, direct_key, exch_hash, fnv1a64, topic_pattern_row, topic_word_offsets)

ONES64 = np.uint64((1 << 64) - 1)


def parse_persist(raw):
    """Packed persist records (PersistHdr + [ex][rk][props][body]) -> [(msg_id, ts_ms, q,
    qpos, expire_ms, ex, rk, props, body)]."""
    raw = np.frombuffer(raw, np.uint8) if isinstance(raw, (bytes, bytearray)) else raw
    hdrs, data_of, off = [], {}, 0
    while off + PERSIST_HDR.itemsize <= len(raw):
        h = raw[off:off + PERSIST_HDR.itemsize].view(PERSIST_HDR)[0]
        b = off + PERSIST_HDR.itemsize
        el, rl, pl, bl = int(h["ex_len"]), int(h["rk_len"]), int(h["props_len"]), int(h["body_len"])
        if int(h["size"]) > PERSIST_HDR.itemsize:   # a message's bytes ride its first record only
            data_of[int(h["msg_id"])] = bytes(raw[b:b + el + rl + pl + bl])
        hdrs.append((h, el, rl, pl))
        if int(h["size"]) <= 0:
            break
        off += int(h["size"])
    out = []
    for h, el, rl, pl in hdrs:
        data = data_of.get(int(h["msg_id"]), b"")
        out.append((int(h["msg_id"]), int(h["ts_ms"]), int(h["q"]), int(h["qpos"]), int(h["expire_ms"]),
                    data[:el], data[el:el + rl], data[el + rl:el + rl + pl], data[el + rl + pl:]))
    return out


def parse_consumed(raw):
    """ConsumedRec[] -> [(msg_id, q, qpos, kind)]."""
    recs = np.frombuffer(bytes(raw), CONSUMED_REC) if isinstance(raw, (bytes, bytearray)) else raw.view(CONSUMED_REC)
    return [(int(r["msg_id"]), int(r["q"]), int(r["qpos"]), int(r["kind"])) for r in recs]


class StepResult:
    __slots__ = ("egress", "ctrl", "txbuf", "events", "segs", "counters", "elapsed")

    def __init__(self):
        self.egress = {}      # conn -> bytes
        self.ctrl = []        # (conn, raw frame bytes of one control command)
        self.txbuf = []       # (conn, wire position, raw bytes): data commands of Tx channels
        self.events = []      # (conn, code, chslot)
        self.segs = []        # (conn, status, consumed, carry, ncmds, err_off)
        self.counters = {}
        self.elapsed = 0.0


class GpuDataPlane(ControlState):
    def __init__(self, device=0, hash_wildcard=True, graph=True, worker=0, default_queue_capacity=1 << 16,
                 world=1, rank=0, shard_map=None, exchanger=None, exchange_lag=0, egress_ref=0, **cfg):
        """``egress_ref``: egress by reference -- a delivery whose body arrived in the
        ingress payload of the same step (or up to ``egress_ref`` steps earlier) is rendered
        without the body, which the host takes from that payload (``finish`` / ``host_egress``
        splice it back in; the native front end sends it with sendmsg iovecs).  The caller
        keeps each payload unchanged until the delivering step's egress is collected
        (``step()`` does: a payload buffer is reused two steps later).  None / -1: off."""
        self.mod = ops.load()
        full = dict(cfg)
        full.setdefault("egress_ref_back", -1 if egress_ref is None else int(egress_ref))
        # (k_frame_scan reads new bytes in place; CHANAMQ_SCAN_IN_PLACE=0 for the copy path)
        full.setdefault("scan_in_place", int(os.environ.get("CHANAMQ_SCAN_IN_PLACE", "1")))
        # per-step IO sets: 3 on a single-GPU engine without the overlapped ingest (the engine
        # keeps 2 otherwise); CHANAMQ_PARITIES=3 selects it (and that engine mode) for tests
        if int(os.environ.get("CHANAMQ_PARITIES", "0")) >= 3 and world == 1:
            full.setdefault("parities", 3)
            full.setdefault("overlap", 0)
        # CHANAMQ_H2D_HSA=1: ingress payloads through HSA, waited for on the device (engine cfg
        # h2d_hsa; single GPU without the overlapped ingest, HSA egress)
        if int(os.environ.get("CHANAMQ_H2D_HSA", "0")) and world == 1:
            full.setdefault("h2d_hsa", 1)
            full.setdefault("overlap", 0)
            full.setdefault("copy_engine", 3)
        full.update(device=device, hash_wildcard=int(hash_wildcard), graph=int(graph), world=world, rank=rank,
                    exchange_lag=int(exchange_lag))
        self.eng = self.mod.Engine(full)
        self.info = self.eng.info()
        sz = self.info["sizeof"]
        assert sz["SegIn"] == SEG_IN.itemsize and sz["SegOut"] == SEG_OUT.itemsize
        assert sz["CtrlRec"] == CTRL_REC.itemsize and sz["ConnOut"] == CONN_OUT.itemsize
        self.device = device
        self.worker = worker
        self.step_no = 0
        i = self.info
        self.carry = np.zeros(i["c_max"], np.int64)
        self._io = [dict(seg_out=self.eng.host_view(f"seg_out{p}").view(SEG_OUT),
                         ctrl_rec=self.eng.host_view(f"ctrl_rec{p}").view(CTRL_REC),
                         conn_out=self.eng.host_view(f"conn_out{p}").view(CONN_OUT),
                         ctrl=self.eng.host_view(f"ctrl{p}")) for p in range(i.get("parities", 2))]
        self.parities = i.get("parities", 2)
        # rendered egress: the engine rotates i["egress_slots"] buffers over the steps
        self._egress = [self.eng.host_view(f"egress_host{e}") for e in range(i["egress_slots"])]
        self._pin = [None] * self.parities
        self.exchanger = exchanger
        self._get_consumed = []   # store records of Basic.Get, emitted with the next step's
        self._pending = None
        self._xprev = None        # parity of the launched step whose exchange is still due
        self.lag = False
        self.native_xchg = bool(i.get("native_xchg"))
        if world > 1 and self.native_xchg:
            # the engine owns the exchange buffers and moves them itself (RCCL / shared
            # memory) under the native front end's sharded stepper (frontend.cpp)
            self.lag = True
        elif world > 1:
            # exchange operands live in torch's allocator so RCCL can use them directly
            import torch
            dev = torch.device("cuda", device)
            u8 = torch.uint8
            self.lag = bool(i["exchange_lag"])
            nb = 2 if self.lag else 1
            self._xs = [(torch.empty(i["xfer_desc_max"] * RDESC.itemsize, dtype=u8, device=dev),
                         torch.empty(i["xfer_bytes"], dtype=u8, device=dev)) for _ in range(nb)]
            self._xr = [(torch.empty(i["import_max"] * RDESC.itemsize, dtype=u8, device=dev),
                         torch.empty(i["xfer_bytes"], dtype=u8, device=dev)) for _ in range(nb)]
            if self.lag:   # parity p packs into S[p] and imports R[p^1] (the previous step's exchange)
                for p in (0, 1):
                    self.eng.set_xfer_parity(p, self._xs[p][0].data_ptr(), self._xs[p][1].data_ptr(),
                                             self._xr[p ^ 1][0].data_ptr(), self._xr[p ^ 1][1].data_ptr())
            else:
                self.eng.set_xfer_buffers(self._xs[0][0].data_ptr(), self._xs[0][1].data_ptr(),
                                          self._xr[0][0].data_ptr(), self._xr[0][1].data_ptr())
        self._deleted_rings = {}
        super().__init__(c_max=i["c_max"], chpc=i["chpc"], q_max=i["q_max"], x_max=i["x_max"],
                         cons_max=i["cons_max"], hash_wildcard=hash_wildcard, ring_pool=i["ring_pool"],
                         default_queue_capacity=default_queue_capacity, world=world, rank=rank,
                         shard_map=shard_map)

    # ================================================================== uploads
    # ``defer`` (set by the broker around control work done while steps keep running): table
    # writes are staged in the engine and ridden by the next submitted step -- applied by
    # its first kernel before it reads anything -- instead of synchronous copies that need
    # the pipeline drained.  Device reads are refused meanwhile (the state they would see
    # is neither before nor after the staged writes).
    defer = False

    def _write(self, name, a, offset):
        if self.defer:
            self.eng.stage_write(name, a, offset)
        else:
            self.eng.upload(name, a, offset)

    def _quiet(self, what):
        if self.defer:
            raise RuntimeError(f"{what}: a device read while control writes are deferred")

    def flush_deltas(self):
        """Apply the staged control writes now (the caller holds the engine: no step in flight)."""
        self.eng.flush_deltas()

    def set_deliver_cap_bytes(self, n):
        """Per-step byte cap of one consumer's deliveries (StepIn.dcap_bytes; 0 = off)."""
        self.eng.set_deliver_cap_bytes(int(n))

    def deltas_pending(self):
        """(records, bytes, channels to mark) staged and not yet taken by a step."""
        return tuple(self.eng.deltas_pending())

    def _up(self, name, arr, index=0):
        a = np.ascontiguousarray(arr)
        self._write(name, a, index * a.itemsize if a.ndim else index * a.itemsize)

    def _up_at(self, name, value, index, dtype):
        a = np.array([value], dtype=dtype)
        self._write(name, a, index * a.itemsize)

    def routing_changed(self):
        i = self.info
        xh = i["xhash"]
        x_hkey = np.zeros(xh, np.uint64)
        x_hval = np.full(xh, -1, np.int32)
        x_type = np.zeros(self.x_max, np.uint32)
        x_fan_off = np.zeros(self.x_max, np.uint32)
        x_fan_n = np.zeros(self.x_max, np.uint32)
        x_t_off = np.zeros(self.x_max, np.uint32)
        x_t_n = np.zeros(self.x_max, np.uint32)
        fan_q, d_q = [], []
        kpool = bytearray()
        dh = i["dhash"]
        d_key = np.zeros(dh, np.uint64)
        d_exch = np.full(dh, -1, np.int32)
        d_kb_off = np.zeros(dh, np.uint32)
        d_kb_len = np.zeros(dh, np.uint32)
        d_q_off = np.zeros(dh, np.uint32)
        d_q_n = np.zeros(dh, np.uint32)
        tb = []   # (exch, queue, pattern)
        for x in sorted(self.exchanges.values(), key=lambda e: e.slot):
            h = exch_hash(self.vhosts[x.vhost], x.name.encode())
            for j in range(xh):
                s = (h + j) & (xh - 1)
                if x_hval[s] < 0:
                    x_hkey[s] = h
                    x_hval[s] = x.slot
                    break
            else:
                raise ControlError(C.RESOURCE_ERROR, "exchange hash full")
            x_type[x.slot] = C.EXCHANGE_TYPE_ID[x.type]
            if x.type == "fanout":
                qs = sorted({q for q, _ in x.bindings})
                x_fan_off[x.slot] = len(fan_q)
                x_fan_n[x.slot] = len(qs)
                fan_q.extend(qs)
            elif x.type == "direct":
                by_key = defaultdict(list)
                for q, k in x.bindings:
                    if q not in by_key[k]:
                        by_key[k].append(q)
                for k, qs in by_key.items():
                    dk = direct_key(fnv1a64(k), x.slot)
                    for j in range(dh):
                        s = (dk + j) & (dh - 1)
                        if d_exch[s] < 0:
                            break
                    else:
                        raise ControlError(C.RESOURCE_ERROR, "direct binding hash full")
                    d_key[s] = dk
                    d_exch[s] = x.slot
                    d_kb_off[s] = len(kpool)
                    d_kb_len[s] = len(k)
                    kpool += k
                    d_q_off[s] = len(d_q)
                    d_q_n[s] = len(qs)
                    d_q.extend(sorted(qs))
            else:  # topic, headers (routes as topic: ExchangeEntity.scala:149-154)
                x_t_off[x.slot] = len(tb)
                bs = sorted(set(x.bindings))
                x_t_n[x.slot] = len(bs)
                tb.extend((x.slot, q, k) for q, k in bs)
        tbp = i["tb_pad"]
        if len(tb) > i["tb_max"]:
            raise ControlError(C.RESOURCE_ERROR, "too many topic bindings for the GPU table")
        t_queue = np.zeros(tbp, np.uint32)
        t_exch = np.zeros(tbp, np.uint32)
        t_kb_off = np.zeros(tbp, np.uint32)
        t_kb_len = np.zeros(tbp, np.uint32)
        t_flags = np.zeros(tbp, np.uint32)
        t_expect = np.full(tbp, -1, np.int32)
        t_mat = np.zeros((tbp, 256), np.int8)
        t_woff = np.zeros((tbp, 8), np.uint16)
        for n, (xs, q, k) in enumerate(tb):
            row, exp, fl = topic_pattern_row(k, self.hash_wildcard)
            t_queue[n], t_exch[n], t_flags[n], t_expect[n] = q, xs, fl, exp
            t_woff[n] = topic_word_offsets(k)
            t_kb_off[n], t_kb_len[n] = len(kpool), len(k)
            kpool += k
            t_mat[n] = row
        for name, arr in (("x_hkey", x_hkey), ("x_hval", x_hval), ("x_type", x_type),
                          ("x_fan_off", x_fan_off), ("x_fan_n", x_fan_n), ("x_t_off", x_t_off),
                          ("x_t_n", x_t_n), ("d_key", d_key), ("d_exch", d_exch), ("d_kb_off", d_kb_off),
                          ("d_kb_len", d_kb_len), ("d_q_off", d_q_off), ("d_q_n", d_q_n),
                          ("t_queue", t_queue), ("t_exch", t_exch), ("t_kb_off", t_kb_off),
                          ("t_kb_len", t_kb_len), ("t_flags", t_flags), ("t_expect", t_expect),
                          ("t_mat", t_mat), ("t_woff", t_woff),
                          ("t_count", np.array([len(tb), 0, 0, 0], np.uint32))):
            self._up_diff(name, arr)
        if fan_q:
            self._up_diff("fan_q", np.array(fan_q, np.uint32))
        if d_q:
            self._up_diff("d_q", np.array(d_q, np.uint32))
        if kpool:
            self._up_diff("kpool", np.frombuffer(bytes(kpool), np.uint8))

    _route_cache = None

    def _up_diff(self, name, arr):
        """A routing table: only the byte runs that differ from its last upload are written.
        A declare / bind rebuilds every table on the host; staging them whole (MBs with a
        large direct hash) in a light section overflowed the step's delta budget at once, so
        RPC-style churn paused the stepper on every cycle."""
        raw = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
        if self._route_cache is None:
            self._route_cache = {}
        old = self._route_cache.get(name)
        self._route_cache[name] = raw.copy()
        if old is None or len(old) != len(raw):
            self._write(name, raw, 0)
            return
        diff = np.flatnonzero(old != raw)
        if not len(diff):
            return
        cut = np.flatnonzero(np.diff(diff) > 64)   # runs closer than 64 B are written as one
        starts = np.concatenate((diff[:1], diff[cut + 1]))
        ends = np.concatenate((diff[cut], diff[-1:])) + 1
        if len(starts) > 16:   # scattered (e.g. key offsets shifted): one record, first to last
            starts, ends = starts[:1], ends[-1:]
        for a, b in zip(starts.tolist(), ends.tolist()):
            self._write(name, raw[a:b], a)

    def _chmap_row(self, conn):
        size = self.info["chmap_size"]
        row = np.zeros(size, np.uint32)
        c = self.conns.get(conn)
        if c is not None:
            for ch, chan in c.channels.items():
                h = chan_hash(ch)
                for j in range(size):
                    s = (h + j) & (size - 1)
                    if row[s] == 0:
                        row[s] = (ch << 16) | 0x8000 | chan.local
                        break
        self._write("chmap", row, conn * size * 4)

    def connection_changed(self, conn):
        c = self.conns.get(conn)
        self._up_at("conn_vhost", self.vhosts[c.vhost] if c else 0, conn, np.uint32)
        self._up_at("conn_frame_max", c.frame_max if c else 0, conn, np.uint32)
        self._up_at("conn_paused", 0, conn, np.uint32)
        self._up_at("carry_len", 0, conn, np.uint32)
        self.carry[conn] = 0
        if c is None:
            self._up_at("conn_paused", 0, conn, np.uint32)
        self._chmap_row(conn)

    def channel_opened(self, chan):
        s = chan.conn * self.chpc + chan.local
        for name, v, dt in (("ch_next_tag", 1, np.uint64), ("ch_uhead", 1, np.uint64),
                            ("ch_ack_upto", 0, np.uint64), ("ch_req_upto", 0, np.uint64),
                            ("ch_mlo", 0xFFFFFFFF, np.uint32), ("ch_mhi", 0, np.uint32),
                            ("ch_confirm_next", 1, np.uint64), ("ch_confirm", 0, np.uint32),
                            ("ch_pub_cnt", 0, np.uint32), ("ch_pub_fail", 0, np.uint32), ("ch_prefetch", 0, np.uint32),
                            ("ch_global", 0, np.uint32), ("ch_flow", 1, np.uint32),
                            ("ch_num", chan.ch, np.uint32), ("ch_unacked", 0, np.uint32),
                            ("ch_win", 0, np.uint32), ("ch_tx", 0, np.uint32)):
            self._up_at(name, v, s, dt)
        self._chmap_row(chan.conn)

    def channel_changed(self, conn, ch):
        chan = self.channel(conn, ch)
        s = self.chslot(conn, ch)
        self._up_at("ch_confirm", int(chan.confirm), s, np.uint32)
        self._up_at("ch_prefetch", chan.prefetch_count, s, np.uint32)
        self._up_at("ch_global", int(chan.global_), s, np.uint32)
        self._up_at("ch_flow", int(chan.flow), s, np.uint32)
        self._up_at("ch_tx", int(chan.tx), s, np.uint32)

    def channel_closing(self, chan):
        # unacked deliveries of a closing channel go back to their queues (AMQP 0-9-1 §1.8)
        s = chan.conn * self.chpc + chan.local
        self._up_at("ch_req_upto", (1 << 62), s, np.uint64)
        self._mark_dirty(s)
        self._up_at("ch_flow", 0, s, np.uint32)
        c = self.conns[chan.conn]
        saved = c.channels.pop(chan.ch)
        self._chmap_row(chan.conn)
        c.channels[chan.ch] = saved

    def _mark_dirty(self, chslot):
        if self.defer:   # the step's first kernel puts it on the dirty list (device atomics)
            self.eng.stage_mark_dirty(int(chslot))
            return
        flag = np.frombuffer(self.eng.download("ch_dirty", chslot * 4, 4), np.uint32)[0]
        if flag:
            return
        n = int(np.frombuffer(self.eng.download("n_dirty", 0, 4), np.uint32)[0])
        self._up_at("dirty_list", chslot, n, np.uint32)
        self._up_at("n_dirty", n + 1, 0, np.uint32)
        self._up_at("ch_dirty", 1, chslot, np.uint32)

    def queue_declared(self, q):
        self._up_at("q_owner", q.owner, q.slot, np.uint32)
        self._up_at("q_excl", q.exclusive_owner + 1 if q.exclusive_owner >= 0 else 0, q.slot, np.uint32)
        self._up_at("q_durable", int(q.durable), q.slot, np.uint32)
        self._up_at("q_ring_off", q.ring_off, q.slot, np.uint64)
        self._up_at("q_ring_mask", q.capacity - 1, q.slot, np.uint64)
        self._up_at("q_max_cap", q.max_capacity, q.slot, np.uint64)
        self._up_at("q_head", 0, q.slot, np.uint64)
        self._up_at("q_tail", 0, q.slot, np.uint64)
        self._up_at("q_ttl", q.ttl_ms, q.slot, np.int64)
        self._up_at("q_rr", 0, q.slot, np.uint32)
        self._up_at("req_q_n", 0, q.slot, np.uint32)
        self._up_at("q_active", 1, q.slot, np.uint32)
        self._sync_consumers()

    def queue_deleted(self, q):
        self._up_at("q_active", 0, q.slot, np.uint32)
        if self.defer:
            # a light control section (steps running): no device read.  The host's view of
            # the ring is current up to the ring moves it has seen (FE_GROW); a move still in
            # flight reports the range it abandoned, which rings_moved then frees
            self._deleted_rings[q.slot] = (q.ring_off, q.capacity)
            self._sync_consumers()
            return
        # if the device grew the ring since the host last looked, ControlState just freed the
        # abandoned range (free anyway); the live one goes back to the pool too
        off = self._u64("q_ring_off", q.slot)
        cap = self._u64("q_ring_mask", q.slot) + 1
        if (off, cap) != (q.ring_off, q.capacity):
            self._ring_free.setdefault(cap, []).append(off)
        self._sync_consumers()

    def consumers_changed(self, q, cid, removed=False):
        if not removed:
            c = self.consumers[cid]
            tag = c.tag.encode()[:255]
            self._up_at("cons_q", c.queue, cid, np.uint32)
            self._up_at("cons_ch", self.chslot(c.conn, c.ch), cid, np.uint32)
            self._up_at("cons_noack", int(c.no_ack), cid, np.uint32)
            # deferred (light control section, steps running): 2 = active from the step after
            # the one applying it, so no Basic.Deliver overtakes the ConsumeOk (k_stage)
            self._up_at("cons_active", 2 if self.defer else 1, cid, np.uint32)
            self._up_at("cons_unacked", 0, cid, np.uint32)
            self._up_at("cons_tag_off", cid * 256, cid, np.uint32)
            self._up_at("cons_tag_len", len(tag), cid, np.uint32)
            if tag:
                self._write("tpool", np.frombuffer(tag, np.uint8), cid * 256)
        else:
            self._up_at("cons_active", 0, cid, np.uint32)
        self._sync_consumers()

    def _sync_consumers(self):
        q_off = np.zeros(self.q_max, np.uint32)
        q_n = np.zeros(self.q_max, np.uint32)
        flat = []
        for q in sorted(self.queue_by_slot.values(), key=lambda x: x.slot):
            q_off[q.slot] = len(flat)
            q_n[q.slot] = len(q.consumers)
            flat.extend(q.consumers)
        self._up("q_cons_off", q_off)
        self._up("q_cons_n", q_n)
        if flat:
            self._up("q_cons", np.array(flat, np.uint32))

    # ---- host-side queue/channel ops between steps (the plane is idle: step() is synchronous)
    def _u64(self, name, idx):
        self._quiet(name)
        return int(np.frombuffer(self.eng.download(name, idx * 8, 8), np.uint64)[0])

    # ---- persistence (engine built with persist=1)
    def take_persist(self):
        """Persist records of the last finished step: [(msg_id, ts_ms, q, qpos, expire_ms,
        ex, rk, props, body)] — durable queue x persistent message, one per enqueue."""
        c = self.last_counters
        self._check_records(c)
        n = min(c["n_persist"], self.info["persist_max"])
        if not n:
            return []
        raw = self.eng.host_view(f"persist{self.eng.persist_slot(self._last_parity)}")[:c["persist_used"]]
        return parse_persist(raw)

    def _check_records(self, c):
        """The device drops store records past persist_max: never commit a partial step."""
        if c["n_persist_overflow"] or c["n_persist"] > self.info["persist_max"] or \
                c["n_consumed"] > self.info["persist_max"]:
            raise RuntimeError(f"persist record buffer overflow ({c['n_persist']} persist / {c['n_consumed']} "
                               f"consumed records > persist_max {self.info['persist_max']})")

    def take_consumed(self):
        """[(msg_id, q, qpos, kind)] of persistent messages that left durable queues."""
        out, self._get_consumed = self._get_consumed, []
        c = self.last_counters
        self._check_records(c)
        n = min(c["n_consumed"], self.info["persist_max"])
        if not n:
            return out
        return out + parse_consumed(self.eng.host_view(f"consumed{self.eng.persist_slot(self._last_parity)}")[:n * CONSUMED_REC.itemsize])

    def take_link_consumed(self, slots):
        """The last finished step's consumed records of the shadow queues ``slots``
        (parallel/links.py); the per-step buffer is left intact for ``take_consumed``."""
        c = getattr(self, "last_counters", None)
        n = min(c["n_consumed"], self.info["persist_max"]) if c and self.info.get("persist") else 0
        if not n:
            return []
        recs = parse_consumed(self.eng.host_view(f"consumed{self.eng.persist_slot(self._last_parity)}")[:n * CONSUMED_REC.itemsize])
        return [r for r in recs if r[1] in slots]

    def take_persist_raw(self):
        """(packed persist records, ConsumedRec bytes) of the last finished step, as the
        native PersistWorker consumes them."""
        c = getattr(self, "last_counters", None)
        if not c:
            return b"", b""
        self._check_records(c)
        p = self._last_parity
        persist = bytes(self.eng.host_view(f"persist{self.eng.persist_slot(p)}")[:c["persist_used"]]) if c["n_persist"] else b""
        n = min(c["n_consumed"], self.info["persist_max"])
        consumed = bytes(self.eng.host_view(f"consumed{self.eng.persist_slot(p)}")[:n * CONSUMED_REC.itemsize]) if n else b""
        return persist, consumed

    def take_get_consumed(self):
        """Store records of Basic.Get calls since the last call (native front end mode,
        where no Python-run step collects them)."""
        out, self._get_consumed = self._get_consumed, []
        return out

    def basic_get(self, conn, ch, q, no_ack, now_ms=None):
        """Basic.Get between steps (k_basic_get): the head of queue slot ``q`` after the
        TTL skip, with the channel's next delivery tag.  Returns (GetOk + header + body
        frames | None when empty, ready messages left).  Reference FrameStage.scala:1199-1229."""
        now = int(time.time() * 1000) if now_ms is None else int(now_ms)
        s = self.chslot(conn, ch)
        while True:
            st, cnt, frames, tag, mid, qpos, persist, exp = self.eng.basic_get(q, s, int(bool(no_ack)), now)
            self._get_consumed.extend((int(m), int(qq), int(qp), 1) for m, qq, qp in exp)
            if st == 5:   # GET_COLD: the head's body is in the cold store -- read it back
                store = getattr(self, "cold_store", None)
                if store is None or not self.cold_in(store):
                    return None, int(cnt)
                continue
            if st != 2:   # GET_RETRY: 64 expired entries skipped, more at the head
                break
        if st == 1:
            if persist:
                self._get_consumed.append((int(mid), q, int(qpos), 0 if no_ack else 3))
            return bytes(frames), int(cnt)
        if st in (3, 4):
            raise ControlError(C.RESOURCE_ERROR, "basic.get: " + ("message exceeds the get buffer" if st == 3
                                                                 else "channel delivery window full"), 60, 70)
        return None, int(cnt)

    def restore(self, items, now_ms=None):
        """Recovery: enqueue stored messages into their queues in the given order.
        items: [(q_slot, msg_id, ts_ms, expire_ms, ex, rk, props, body, persistent, redelivered)]."""
        now = int(time.time() * 1000) if now_ms is None else int(now_ms)
        if self.lag and not self.native_xchg:   # native: the engine refuses it while an exchange is pending
            raise RuntimeError("restore() would overwrite the lagged exchange's pending imports")
        cap = max(1, min(self.info["restore_max"] or self.info["import_max"], self.info["import_max"]))
        room = self.info["xfer_bytes"]
        chunks, cur, cur_b = [], [], 0
        for it in items:   # batches within the import buffers: records and payload bytes
            b = len(it[4]) + len(it[5]) + len(it[6]) + len(it[7]) + 16
            if cur and (len(cur) == cap or cur_b + b > room):
                chunks.append(cur)
                cur, cur_b = [], 0
            cur.append(it)
            cur_b += b
        if cur:
            chunks.append(cur)
        total = 0
        for chunk in chunks:
            desc = np.zeros(len(chunk), RDESC)
            pay = bytearray()
            for i, (q, mid, ts, exp, ex, rk, props, body, persistent, red) in enumerate(chunk):
                d = desc[i]
                d["pay_off"] = len(pay)
                d["body_len"], d["props_len"], d["exch"] = len(body), len(props), -1
                d["flags"] = MF_RESTORE | (MF_PERSIST if persistent else 0) | (MF_REDELIVERED if red else 0)
                d["ex_len"], d["rk_len"] = len(ex), len(rk)
                d["expire_ms"], d["ts_ms"], d["xid"], d["tq"] = exp, ts, mid, q
                rec = ex + rk + props + body
                pay += rec + b"\0" * ((-len(rec)) % 16)
            total += self.eng.restore(desc.view(np.uint8), np.frombuffer(bytes(pay) or b"\0", np.uint8)[:len(pay)],
                                      now)
        return total

    # ---- messages larger than a connection's carry (host-assembled publishes)
    def take_carry(self, conn):
        """The bytes the device holds for a paused connection (its carry: the frames after
        a command the host took over), removed from the device."""
        self._quiet("carry")
        n = int(np.frombuffer(self.eng.download("carry_len", 4 * conn, 4), np.uint32)[0])
        data = bytes(self.eng.download("carry", conn * self.info["carry_cap"], n)) if n else b""
        self._up_at("carry_len", 0, conn, np.uint32)
        self.carry[conn] = 0
        return data

    def max_host_message(self):
        """Largest message the host-publish path takes: it must fit the restore buffers and
        one step's egress (its Basic.Deliver frames) with room to spare."""
        i = self.info
        return max(0, min(i["xfer_bytes"] - 4096, i["egress_cap"] // 2, i["log_bytes"] // 4))

    def publish_host(self, conn, ch, exch_slot, ex, rk, props, body, flags, expire_ms=0, ts_ms=0, now_ms=None):
        """Enqueue a publish the host assembled (larger than the connection's carry):
        routed on the device by its exchange like any publish, counted for the publisher
        channel's confirms (the next step's Basic.Ack / Nack covers it).  Between steps.
        Returns the number of messages stored (0: unroutable or dropped)."""
        now = int(time.time() * 1000) if now_ms is None else int(now_ms)
        # sharded plane (at a sync point, server/gpu_broker.py _apply_big): stored in this
        # rank's queues only -- imported records are never forwarded; the owners of the
        # other queues enqueue their copies themselves (publish_to_queues)
        desc = np.zeros(1, RDESC)
        d = desc[0]
        d["pay_off"], d["body_len"], d["props_len"], d["exch"] = 0, len(body), len(props), exch_slot
        d["flags"] = MF_HOSTPUB | (flags & (MF_PERSIST | MF_HAS_TS))
        d["ex_len"], d["rk_len"] = len(ex), len(rk)
        d["expire_ms"], d["ts_ms"], d["xid"], d["tq"] = expire_ms, ts_ms, 0, 0
        d["pad"][0] = self.chslot(conn, ch)
        d["pad"][1] = conn
        rec = bytes(ex) + bytes(rk) + bytes(props) + bytes(body)
        pay = np.frombuffer(rec + b"\0" * ((-len(rec)) % 16), np.uint8)
        return self.eng.restore(desc.view(np.uint8), pay, now)

    def publish_to_queues(self, slots, ex, rk, props, body, flags, expire_ms=0, ts_ms=0, now_ms=None):
        """A host-assembled publish into exactly the given local queues (a sharded owner's
        part of a large publish routed on another rank): one MF_ONEQ record per queue,
        each stored with a new message id.  Between steps / at a sync point."""
        now = int(time.time() * 1000) if now_ms is None else int(now_ms)
        if not slots:
            return 0
        desc = np.zeros(len(slots), RDESC)
        rec = bytes(ex) + bytes(rk) + bytes(props) + bytes(body)
        pad = rec + b"\0" * ((-len(rec)) % 16)
        pay = bytearray()
        for i, q in enumerate(slots):
            d = desc[i]
            d["pay_off"], d["body_len"], d["props_len"], d["exch"] = len(pay), len(body), len(props), -1
            d["flags"] = MF_ONEQ | (flags & (MF_PERSIST | MF_HAS_TS))
            d["ex_len"], d["rk_len"] = len(ex), len(rk)
            d["expire_ms"], d["ts_ms"], d["xid"], d["tq"] = expire_ms, ts_ms, 0, int(q)
            pay += pad
        return self.eng.restore(desc.view(np.uint8), np.frombuffer(bytes(pay), np.uint8), now)

    # ---- cold bodies to host memory (built with spill_bytes > 0)
    def spill(self, frac=0.5, hot=1024):
        """Move cold message bodies to the host spill ring (between steps): queued
        messages whose slot lies in the oldest ``frac`` of the HBM log (but the first
        ``hot`` of a queue with consumers).  Returns the bytes moved; the log tail advances
        over the emptied blocks at the next step."""
        if not self.info.get("spill_bytes"):
            return 0
        tail = self._u64("log_tail", 0)
        return int(self.eng.spill(int(tail + frac * self.info["log_bytes"]), int(hot)))

    # ---- cold store: the third body tier (store/cold.py; built with spill_bytes > 0)
    def cold_out(self, store, hot=1 << 16, max_bytes=256 << 20, frac=0.5):
        """Spilled bodies of single-queue non-persistent messages in the oldest ``frac``
        of the spill ring (the ring frees from its tail) go to ``store`` (between steps),
        but not the first ``hot`` entries of a queue with consumers; returns the bytes
        moved.  Their queues then hold deliveries at the first cold position until
        ``cold_in`` reads them back."""
        from ..store.cold import COLD_REC
        if not self.info.get("spill_bytes"):
            return 0
        lim = int(frac * self.info["spill_bytes"])   # (from the ring's tail)
        recs = np.frombuffer(self.eng.cold_pick(int(hot), lim, 1 << 16, int(max_bytes)), COLD_REC).copy()
        recs = self._cold_store(store, recs)
        if recs is None:
            return 0
        self.eng.cold_commit(recs)
        return int(recs["bytes"].sum())

    def _cold_store(self, store, recs):
        recs = recs[recs["bytes"] > 0]
        if not len(recs):
            return None
        ring, sb = self._spill_view(), self.info["spill_bytes"]
        views = [memoryview(ring[int(p) % sb:int(p) % sb + int(n)]) for p, n in zip(recs["pos"], recs["bytes"])]
        recs["cold"] = store.put_many(views)
        return recs

    def _cold_load(self, store, recs):
        ring, sb = self._spill_view(), self.info["spill_bytes"]
        for p, n, c in zip(recs["pos"], recs["bytes"], recs["cold"]):
            if n:
                store.get_into(int(c), memoryview(ring[int(p) % sb:int(p) % sb + int(n)]))

    # ---- the cold tier beside the steps (single GPU, pipelined front end): ``run(post)``
    # posts one engine side operation, gets a step to carry it and returns its result
    # (GpuBroker._side).  No pipeline drain: the steps keep running while the store is
    # written or read.
    def cold_out_side(self, store, run, hot=1 << 16, max_bytes=256 << 20, frac=0.5, min_used=0.6):
        """cold_out with the pick and the commit as side operations; nothing moves while
        the spill ring is less than ``min_used`` full (checked on the device)."""
        from ..store.cold import COLD_REC
        sb = self.info.get("spill_bytes")
        if not sb:
            return 0
        raw = run(lambda: self.eng.side_cold_pick(int(hot), int(frac * sb), int(min_used * sb), 1 << 16,
                                                  int(max_bytes)))
        recs = self._cold_store(store, np.frombuffer(raw, COLD_REC).copy())
        if recs is None:
            return 0
        run(lambda: self.eng.side_cold_commit(recs))
        return int(recs["bytes"].sum())

    def cold_in_side(self, store, run, window=1 << 15):
        """cold_in with the scan and the switch-back as side operations."""
        from ..store.cold import COLD_REC
        if not self.info.get("spill_bytes"):
            return 0
        recs = np.frombuffer(run(lambda: self.eng.side_cold_scan(int(window), 1 << 16)), COLD_REC).copy()
        self._cold_load(store, recs)
        run(lambda: self.eng.side_cold_in(recs))
        return int(recs["bytes"].sum())

    def cold_live_side(self, run):
        return np.frombuffer(run(self.eng.side_cold_live), np.int64).copy()

    def cold_in(self, store, window=1 << 15):
        """Bodies of cold entries within ``window`` positions of their queue's head read
        back into the spill ring (between steps); returns the bytes moved."""
        from ..store.cold import COLD_REC
        if not self.info.get("spill_bytes"):
            return 0
        recs = np.frombuffer(self.eng.cold_scan(int(window), 1 << 16), COLD_REC).copy()
        self._cold_load(store, recs)
        self.eng.cold_in(recs)
        return int(recs["bytes"].sum())

    def cold_live(self):
        return np.frombuffer(self.eng.download("cold_live"), np.int64)

    def _spill_view(self):
        v = getattr(self, "_spill_hv", None)
        if v is None:
            v = self._spill_hv = self.eng.host_view("spill")
        return v

    def spill_used(self):
        """Bytes between the spill ring's tail and head (live + not yet reclaimed)."""
        if not self.info.get("spill_bytes"):
            return 0
        return self._u64("spill_head", 0) - self._u64("spill_tail", 0)

    ID_SLOT_BITS = 18   # dp_state.h: snowflake id slots per millisecond (64 worker ids x 4096)

    def seed_ids(self, min_ms):
        """Recovery: new snowflake ids start at millisecond >= ``min_ms`` (above every
        recovered id), whatever the wall clock says."""
        cur = self._u64("id_next", 0)
        want = int(min_ms) << self.ID_SLOT_BITS
        if want > cur:
            self._up_at("id_next", want, 0, np.uint64)

    @staticmethod
    def id_group_workers(group):
        """Worker ids (10-bit snowflake field) owned by GPU id group ``group``."""
        return list(range(group * 64, group * 64 + 64))

    def memory_in_use(self):
        """Body-log slot bytes held by live messages (after the last finished step)."""
        c = getattr(self, "last_counters", None)
        return int(c["live_bytes"]) if c else 0

    def message_count(self, q):
        """Ready messages of queue slot ``q`` (AMQP Queue.DeclareOk message-count)."""
        return self._u64("q_tail", q) - self._u64("q_head", q)

    def queue_tail(self, q):
        """Queue position the next enqueue into slot ``q`` gets."""
        return self._u64("q_tail", q)

    def purge(self, q):
        """Queue.Purge: mark every ready entry expired; the next step's dequeue (K12 TTL
        skip) releases them and their body-log bytes.  Returns the purged count."""
        head, tail = self._u64("q_head", q), self._u64("q_tail", q)
        n = tail - head
        if n <= 0:
            return 0
        qq = self.queue_by_slot[q]
        self._refresh_ring(qq)
        mask = qq.capacity - 1
        base = qq.ring_off * 16
        for lo in range(head, tail, mask + 1):
            k = min(tail - lo, mask + 1)
            i0 = lo & mask
            first = min(k, mask + 1 - i0)
            for start, cnt in ((i0, first), (0, k - first)):
                if cnt <= 0:
                    continue
                raw = np.frombuffer(self.eng.download("ring", base + start * 16, cnt * 16), np.uint8).copy()
                ent = raw.view(np.int64).reshape(cnt, 2)
                ent[:, 1] = 1   # expire_ms = 1 ms after the epoch
                self.eng.upload("ring", raw, base + start * 16)
        return n

    def apply_ack(self, conn, ch, tag, multiple=False, requeue=False, kind="ack"):
        """Basic.Ack / Nack / Reject applied between steps (Tx.Commit of a transactional
        channel): the same marks k_decode makes; k_chan_advance resolves them next step."""
        s = self.chslot(conn, ch)
        nt = self._u64("ch_next_tag", s)
        requeue = bool(requeue) and kind != "ack"
        if tag == 0 and multiple:
            tag = nt - 1
        if multiple:
            name = "ch_req_upto" if requeue else "ch_ack_upto"
            if tag > self._u64(name, s):
                self._up_at(name, tag, s, np.uint64)
        elif self._u64("ch_uhead", s) <= tag < nt:
            ucap = self.info["ucap"]
            off = (s * ucap + ((tag - 1) & (ucap - 1))) * USLOT.itemsize
            st = int(np.frombuffer(self.eng.download("uwin", off, 4), np.uint32)[0])
            if st == US_PENDING:
                self._up_at("uwin", US_REQUEUE if requeue else US_ACKED, off // 4, np.uint32)
        self._mark_dirty(s)

    def recover(self, conn, ch):
        """Basic.Recover(requeue): requeue every outstanding delivery of the channel."""
        s = self.chslot(conn, ch)
        upto = max(self._u64("ch_req_upto", s), self._u64("ch_next_tag", s) - 1)
        self._up_at("ch_req_upto", upto, s, np.uint64)
        self._mark_dirty(s)

    def unpause(self, conn):
        """The connection's bytes are processed again from the next submitted step (k_stage
        clears the device flag): safe from any thread while steps are in flight."""
        c = self.conns.get(conn)
        if c is not None:
            c.paused = False
        self.eng.stage_unpause(int(conn))

    # ================================================================== steps
    def _pinned(self, n, parity):
        pin = self._pin[parity]
        if pin is None or len(pin) < n:
            pin = self._pin[parity] = self.mod.alloc_pinned(max(n, 1 << 20))
        return pin

    def step(self, inputs=None, now_ms=None, collect=True, with_carry=True):
        """One synchronous data-plane step.  ``inputs``: {conn: bytes}.  Connections
        holding carry (partial commands) are re-presented once unpaused (``with_carry``;
        off when the native front end owns the other connections' bytes)."""
        segs, ptr, n = self.stage(inputs, with_carry)
        return self.step_raw(segs, ptr, n, now_ms, collect)

    def stage(self, inputs, with_carry=True):
        """{conn: bytes} (+ connections holding carry) -> (SegIn[], pinned ptr, bytes)."""
        inputs = inputs or {}
        conns = set(inputs)
        for c in np.nonzero(self.carry)[0] if with_carry else ():
            c = int(c)
            if c in self.conns and not self.conns[c].paused:
                conns.add(c)
        order = sorted(conns)
        segs = np.zeros(len(order), SEG_IN)
        total = sum((len(inputs.get(c, b"")) + 15) & ~15 for c in order)
        pin = self._pinned(total + 16, self.step_no % self.parities)
        off = 0
        for k, c in enumerate(order):
            data = inputs.get(c, b"")
            n = len(data)
            if n:
                pin[off:off + n] = np.frombuffer(data, np.uint8)
            segs[k] = (c, n, off)
            off += (n + 15) & ~15
        return segs, pin.ctypes.data, off

    def step_raw(self, segs, payload_ptr, payload_len, now_ms=None, collect=True):
        t = self.submit_raw(segs, payload_ptr, payload_len, now_ms)
        return self.finish(t, collect=collect)

    def xchg_setup(self, kind, arg, members, timeout_ms=10000, failover=False, counts_shm="", async_x=False):
        """Native exchange backend over the live ranks ``members``: "rccl" (arg = the
        128-byte unique id from ``xchg_unique_id()``) or "shm" (arg = a shared-memory name
        common to the group, for ranks sharing one host).  ``counts_shm`` (rccl): move the
        per-step counts through host shared memory (ranks of one node), the bulk on RCCL.
        ``async_x``: each step's exchange runs on the engine's exchange thread and phase B
        waits for it on the device; ``exchange()`` returns the previous step's result."""
        self.eng.xchg_setup(kind, arg, sorted(int(m) for m in members), int(timeout_ms), bool(failover),
                            counts_shm, bool(async_x))

    def xchg_unique_id(self):
        return self.mod.Engine.xchg_unique_id()

    # ---- remote-consumer links on the device (parallel/links.py DeviceLinks)
    def set_link_queue(self, slot, owner):
        """Connection side: consumption of shadow queue ``slot`` acks at rank ``owner``
        (None: no acks)."""
        self._up_at("q_link_owner", 0 if owner is None else int(owner) + 1, slot, np.uint32)

    def set_link_conn(self, pc, dest, tq, epoch):
        """Owner side: pseudo connection ``pc`` ships its deliveries to rank ``dest`` as
        restore records for shadow slot ``tq``; acks for ``tq`` settle its channel 1."""
        self._up_at("conn_link", int(dest) + 1, pc, np.uint32)
        self._up_at("conn_link_tq", tq, pc, np.uint32)
        self._up_at("conn_link_epoch", epoch, pc, np.uint32)
        self._up_at("q_link_ch", self.chslot(pc, 1), tq, np.uint32)
        self._up_at("q_link_epoch", epoch, tq, np.uint32)

    def clear_link_conn(self, pc, tq):
        self._up_at("conn_link", 0, pc, np.uint32)
        self._up_at("q_link_ch", 0xFFFFFFFF, tq, np.uint32)

    def set_link_conns(self, conns):
        a = np.zeros(64, np.uint32)
        a[:len(conns)] = conns
        self._up("link_conns", a)
        self._up_at("n_link_conns", len(conns), 0, np.uint32)

    # ---- unbounded queues: the device grows rings (k_ring_plan); the host mirrors it
    _deleted_rings = None
    _ring_chunk = (0, 0)

    def _ring_alloc(self, cap):
        """Rings come from one pool whose bump pointer lives on the device (k_ring_plan
        allocates from it mid-step); ranges returned by deletes / growth are reused first.
        In a light control section (steps running, no device reads) a new ring comes from
        the host's reserved chunk (``reserve_ring_chunk``)."""
        lst = self._ring_free.get(cap)
        if lst:
            return lst.pop()
        off, left = self._ring_chunk
        if left >= cap:
            self._ring_chunk = (off + cap, left - cap)
            return off
        if self.defer:
            raise ControlError(C.RESOURCE_ERROR, "ring chunk exhausted in a light section")
        top = self._u64("ring_top", 0)
        if top + cap > self.ring_pool and left and off + left == top:
            top, self._ring_chunk = off, (0, 0)   # the unused light-section chunk goes back first
        if top + cap > self.ring_pool:
            raise ControlError(C.RESOURCE_ERROR, "ring pool exhausted")
        self._up_at("ring_top", top + cap, 0, np.uint64)
        return top

    def reserve_ring_chunk(self, entries):
        """(Steps paused / between steps) take ``entries`` ring entries from the device's bump
        pointer for queues declared in light sections (what is left of the last chunk goes
        back to the free lists).  Returns the entries now reserved."""
        off, left = self._ring_chunk
        if left >= entries // 2:
            return left
        top = self._u64("ring_top", 0)
        if left and off + left == top:   # the old remainder is the pool's top: extend it in place
            top, left = off, 0
        # (at most an eighth of what is left: the device grows rings from the same pool mid-step)
        take = min(int(entries), (self.ring_pool - top) // 8)
        if take <= 0:
            return self._ring_chunk[1]   # (nothing changed)
        self._up_at("ring_top", top + take, 0, np.uint64)
        if left:   # (power-of-two pieces of the old remainder to the free lists)
            while left:
                k = 1 << (left.bit_length() - 1)
                self._ring_free.setdefault(k, []).append(off)
                off, left = off + k, left - k
        self._ring_chunk = (top, take)
        return take

    def ring_light_ok(self, cap):
        """A ring of ``cap`` entries can be allocated without a device read."""
        return bool(self._ring_free.get(cap)) or self._ring_chunk[1] >= cap

    def _refresh_ring(self, q):
        """The device may have moved the queue's ring: adopt its current one and return the
        range the host knew to the pool."""
        off = self._u64("q_ring_off", q.slot)
        cap = self._u64("q_ring_mask", q.slot) + 1
        if (off, cap) != (q.ring_off, q.capacity):
            self._ring_free.setdefault(q.capacity, []).append(q.ring_off)
            q.ring_off, q.capacity = off, cap

    def rings_moved(self, raw):
        """RingMove records of a finished step (or the front end's FE_GROW event)."""
        for mv in np.frombuffer(raw, RING_MOVE):
            dr = (self._deleted_rings or {}).get(int(mv["q"]))
            if dr is not None and dr == (int(mv["old_off"]), int(mv["old_mask"]) + 1):
                # the queue was deleted in a light section while this move was in flight: its
                # old range went back with the delete, the new one goes now
                del self._deleted_rings[int(mv["q"])]
                self._ring_free.setdefault(int(mv["new_mask"]) + 1, []).append(int(mv["new_off"]))
                continue
            q = self.queue_by_slot.get(int(mv["q"]))
            if q is not None and q.owner == self.rank and q.ring_off == int(mv["old_off"]):
                self._ring_free.setdefault(q.capacity, []).append(q.ring_off)
                q.ring_off, q.capacity = int(mv["new_off"]), int(mv["new_mask"]) + 1

    def submit_raw(self, segs, payload_ptr, payload_len, now_ms=None):
        """Asynchronous half of a step: returns a ticket for ``finish``.  At most two
        steps may be outstanding (double-buffered step IO)."""
        now = int(time.time() * 1000) if now_ms is None else int(now_ms)
        t0 = time.perf_counter()
        if len(segs):   # the device stages every segment's carry in front of its new bytes
            staged = int(self.carry[segs["conn"]].sum()) + 48 * len(segs)
            if staged > self.info["carry_budget"]:
                raise RuntimeError(f"step carries {staged} B > carry_budget {self.info['carry_budget']} B")
        if self.world > 1 and self.native_xchg:
            # a step run by the control plane at a synchronisation point (no exchange
            # pending on any rank): phase A, no exchange (it carries no client bytes that
            # could route to another rank), phase B
            if len(segs):
                raise RuntimeError("host-run steps of a sharded node carry no client bytes")
            # SF_NODISPATCH: nothing is delivered or shipped to links (it could not travel)
            p = self.eng.submit(segs, int(payload_ptr), int(payload_len), now, self.step_no, now, self.worker,
                                False, 1)
            self.step_no += 1
            self.eng.drop_exchange(p)
            self.eng.launch_b(p)
            return (p, len(segs), t0, self.eng.egress_slot(p))
        if self.world > 1 and self.lag and self.exchanger is not None:
            # one process per rank, pipelined exchange: queue H2D(t), then run step t-1's
            # all-to-all while those bytes cross PCIe, then launch step t (whose phase B
            # imports t-1's exchange) -- the host never waits on H2D(t) + phase A(t)
            p = self.eng.submit(segs, int(payload_ptr), int(payload_len), now, self.step_no, now, self.worker,
                                True)
            self.step_no += 1
            if self._xprev is not None:
                self._exchange_parity(self._xprev)
            self.eng.launch(p)
            self._pending = self._xprev = p
            return (p, len(segs), t0, self.eng.egress_slot(p))
        p = self.eng.submit(segs, int(payload_ptr), int(payload_len), now, self.step_no, now, self.worker)
        self.step_no += 1
        if self.world > 1:
            self._pending = p
            cnt = self.eng.send_counts(p)
            if cnt[-1]:
                raise RuntimeError("cross-rank send buffers overflowed (xfer_desc_max / xfer_bytes)")
            self._send_counts = cnt[:-1]
            if self.exchanger is not None:   # one process per rank: collective now
                recv = self.exchanger.exchange(self._send_counts, self.xfer_send_desc(), self.xfer_send_pay(),
                                               self.xfer_recv_desc(), self.xfer_recv_pay())
                if self.lag:
                    self.set_import(recv)
                else:
                    self.submit_b(recv)
        return (p, len(segs), t0, self.eng.egress_slot(p))

    def prefetch(self, payload_ptr, payload_len):
        """Queue the NEXT step's ingress payload H2D now (overlapped single-GPU engine): it
        crosses PCIe while the current steps run; that step must then be submitted with the
        same payload.  Returns False when not applicable (nothing queued)."""
        return bool(self.eng.prefetch(int(payload_ptr), int(payload_len)))

    def submit_lockstep(self, segs, payload_ptr, payload_len, now_ms=None):
        """One lockstep step of a sharded plane on the engine's native exchange (RCCL over
        xGMI, or host shared memory), in the order the native front end's sharded stepper
        runs it (frontend.cpp ``stepper_sharded``): H2D(t) and phase A(t) are queued, then
        the previous step's exchange runs on the exchange stream while A(t) executes, then
        phase B(t) -- which imports that exchange -- is queued behind it.  The host only
        blocks in the count exchange (``counts_shm``: a shared-memory barrier)."""
        if not (self.world > 1 and self.native_xchg):
            raise RuntimeError("submit_lockstep: needs a sharded plane built with native_xchg=1")
        now = int(time.time() * 1000) if now_ms is None else int(now_ms)
        t0 = time.perf_counter()
        p = self.eng.submit(segs, int(payload_ptr), int(payload_len), now, self.step_no, now, self.worker)
        self.step_no += 1
        q = self._xprev
        if q is not None:
            rc, _ = self.eng.exchange(q, 0)
            if rc != 0:
                self.eng.drop_exchange(q)
                raise RuntimeError(f"rank {self.rank}: native exchange failed (rc {rc}: a peer did not answer)")
        self.eng.launch_b(p)
        self._xprev = p
        return (p, len(segs), t0, self.eng.egress_slot(p))

    def _exchange_parity(self, q):
        """All-to-all of the launched step of parity ``q`` (its phase A packed S[q]; the
        received records land in R[q], imported by the next launched step)."""
        cnt = self.eng.send_counts(q)
        if cnt[-1]:
            raise RuntimeError("cross-rank send buffers overflowed (xfer_desc_max / xfer_bytes)")
        self._send_counts = cnt[:-1]
        recv = self.exchanger.exchange(self._send_counts, self._xs[q][0], self._xs[q][1],
                                       self._xr[q][0], self._xr[q][1])
        self.set_import(recv)

    # ---- sharded step, phase B (LocalCluster drives it after its in-process exchange)
    def pending_send_counts(self):
        return self._send_counts

    # exchange operands of the step in flight (lag: S[p] -> R[p], imported by the next step)
    def _xp(self):
        return self._pending if self.lag else 0

    def xfer_send_desc(self):
        return self._xs[self._xp()][0]

    def xfer_send_pay(self):
        return self._xs[self._xp()][1]

    def xfer_recv_desc(self):
        return self._xr[self._xp()][0]

    def xfer_recv_pay(self):
        return self._xr[self._xp()][1]

    def set_import(self, recv):
        """exchange_lag: this step's exchange is complete on the current torch stream; the
        next step's phase B imports it."""
        import torch
        stream = torch.cuda.current_stream(self.device).cuda_stream
        self.eng.set_import([int(x) for x in recv], int(stream))

    def submit_b(self, recv):
        import torch
        stream = torch.cuda.current_stream(self.device).cuda_stream
        self.eng.submit_b(self._pending, [int(x) for x in recv], int(stream))
        self._pending = None

    def wait(self, ticket):
        """The blocking half of ``finish``: returns once the step's kernels are done and its
        parity is free for the next submit; ``finish(ticket, waited=True)`` then collects.  A
        driver that submits between the two puts the next step's ingress H2D right behind
        the wait instead of behind the previous step's bookkeeping."""
        self.eng.wait_results(ticket[0])

    def finish(self, ticket, collect=True, wait_egress=True, collect_egress=True, waited=False):
        p, nseg, t0, slot = ticket
        if not waited:
            self.eng.wait_results(p)
        self._last_parity = p
        res = StepResult()
        res.counters = c = self.eng.counters(p)
        self.last_counters = c
        if c["n_grow"]:
            self.rings_moved(self.eng.host_view(f"grow{p}")[:RING_MOVE.itemsize * min(c["n_grow"], 4096)].tobytes())
        io = self._io[p]
        so = io["seg_out"][:nseg]
        self.carry[so["conn"]] = so["carry"]
        paused = (so["status"] & SS_CTRL) != 0
        if paused.any():
            for conn in so["conn"][paused]:
                cc = self.conns.get(int(conn))
                if cc is not None:
                    cc.paused = True
        self.eng.egress_copy(p)
        if collect:
            res.segs = [tuple(int(x) for x in (r["conn"], r["status"], r["consumed"], r["carry"],
                                                 r["ncmds"], r["err_off"])) for r in so]
            nctrl = min(c["n_ctrl"], len(io["ctrl_rec"]))
            for rec in io["ctrl_rec"][:nctrl]:
                if int(rec["off"]) == INVALID:
                    res.events.append((int(rec["conn"]), int(rec["len"]), int(rec["seg"])))
                else:
                    o, n, sg = int(rec["off"]), int(rec["len"]), int(rec["seg"])
                    if sg & CTRL_TXBUF:
                        res.txbuf.append((int(rec["conn"]), sg & ~CTRL_TXBUF, bytes(io["ctrl"][o:o + n])))
                    elif sg & CTRL_DGET:   # (the connection was not paused)
                        res.ctrl.append((int(rec["conn"]), bytes(io["ctrl"][o:o + n]), True))
                    else:
                        res.ctrl.append((int(rec["conn"]), bytes(io["ctrl"][o:o + n])))
            res.txbuf.sort()
        if wait_egress or collect:
            self.eng.egress_wait_slot(slot)
        if collect and collect_egress:
            eg, co = self._wire(self._egress[slot], io["conn_out"], c)
            for conn in np.nonzero(co["len"])[0]:
                o, n = int(co["off"][conn]), int(co["len"][conn])
                res.egress[int(conn)] = bytes(eg[o:o + n])
        res.elapsed = time.perf_counter() - t0
        return res

    def _wire(self, eg, co, c):
        """The step's egress as sent on the wire: with referenced bodies (Counters.n_ref)
        the rendered bytes with every body spliced in from its host ingress payload at its
        gather entry (EgressRef), and the connections' (offset, length) in that buffer."""
        if not c["n_ref"]:
            return eg, co
        n = min(int(c["n_deliv"]), int(self.info["deliv_max"]))
        go = int(c["gath_off"])
        tab = eg[go:go + 16 * n].view(EGRESS_REF)
        refs = tab[tab["len"] > 0].copy()
        dst, ln = refs["dst"].astype(np.int64), refs["len"].astype(np.int64)
        out = np.empty(go + int(ln.sum()), np.uint8)
        prev = w = 0
        for d, src, k in zip(dst.tolist(), refs["src"].tolist(), ln.tolist()):
            out[w:w + d - prev] = eg[prev:d]
            w += d - prev
            ctypes.memmove(out.ctypes.data + w, src, k)
            w += k
            prev = d
        out[w:w + go - prev] = eg[prev:go]
        cum = np.concatenate([[0], np.cumsum(ln)])
        off, cl = co["off"].astype(np.int64), co["len"].astype(np.int64)
        s0 = cum[np.searchsorted(dst, off, side="left")]
        s1 = cum[np.searchsorted(dst, off + cl, side="left")]
        wco = np.zeros(len(co), CONN_OUT)
        wco["off"], wco["len"] = off + s0, cl + (s1 - s0)
        return out, wco

    def host_egress(self, ticket):
        """(egress bytes, ConnOut) of a finished step as sent on the wire: zero-copy views
        when no delivery referenced a host body, else a spliced copy (``_wire``)."""
        io = self._io[ticket[0]]
        return self._wire(self._egress[ticket[3]], io["conn_out"], self.eng.counters(ticket[0]))

    def step_done(self, ticket):
        """Non-blocking: the step's kernels have finished (``finish`` will not wait)."""
        return bool(self.eng.step_done(ticket[0]))

    def egress_done(self, ticket):
        """Non-blocking: the finished step's egress bytes are in host memory."""
        return bool(self.eng.egress_done_slot(ticket[3]))

    def egress_wait(self, ticket):
        # by the slot the step rendered into (recorded at submit): a later step of the same
        # parity has its own slot, so waiting "by parity" would wait for the wrong copy
        self.eng.egress_wait_slot(ticket[3])
