"""AMQP 0-9-1 server whose data path is the GPU data plane.

Sockets, the connection handshake and control methods are handled on the host; once a
connection is open every byte it sends goes into the next data-plane step, which scans
frames, routes/stores/enqueues publishes, processes acks, dispatches deliveries and
renders the egress bytes (csrc/kernels/dataplane.hip).  The device pauses a connection
at its first control command and hands the raw command back; this module executes it
against ``ControlState`` (which pushes the changed tables to the device), writes the
reply, and unpauses the connection, so per-connection ordering is exactly the wire order
(the reference's FrameStage does the same per connection: chana-mq-server/src/main/
scala/chana/mq/amqp/server/engine/FrameStage.scala:319-500).

The plane can be a ``GpuDataPlane`` (HIP) or a ``GoldenDataPlane`` (CPU executable
spec, used by the CPU tests of this server).

Basic.Get: with the pipelined front end it is served inside the next step (k_dequeue,
staged by the front end; the broker handles Get and its answer without pausing the
stepper); the other front ends run it between steps (k_basic_get).  Transactions: on a Tx
channel the device hands publishes / acks to the host instead of applying them
(CK_TXBUF); Tx.Commit applies the acks between steps and injects the publishes through a
pseudo-connection in the next step, Tx.Rollback drops them.  Not on the GPU path yet
(540 NOT_IMPLEMENTED; the host-path broker in csrc/core serves it): Exchange.Bind/Unbind.
Sharded: consumers and Basic.Get may name a queue another rank owns (parallel/links.py).
"""

import collections
import logging
import os
import selectors
import socket
import struct
import threading
import time
import uuid

import numpy as np

from ..engine.control import ControlError, normalize_vhost
from ..engine.layout import MF_HAS_TS, MF_PERSIST, SS_FRAME_ERROR, SS_OVERFLOW, SS_TOO_LARGE, SS_UNEXPECTED
from ..protocol import constants as C
from ..protocol.codec import (Method, decode_content_header, decode_method, encode_method_frame, encode_table,
                              render_command)

HEARTBEAT = C.HEARTBEAT_FRAME
_REPLICATED_METHODS = {"exchange.declare", "exchange.delete", "queue.declare", "queue.bind", "queue.unbind",
                       "queue.delete"}
_STORED_METHODS = _REPLICATED_METHODS


class _Conn:
    __slots__ = ("sock", "id", "state", "inbuf", "out", "frame_max", "heartbeat", "last_rx", "last_tx",
                 "closing_channels", "last_queue", "peer", "user", "cap_blocked", "big", "big_rest")

    def __init__(self, sock, cid, peer):
        self.sock, self.id, self.peer = sock, cid, peer
        self.state = "header"   # header -> start -> tune -> open (<-> bigpub [-> bigwait]) -> closing -> closed
        self.big = None         # a publish larger than the device carry being assembled on the host
        self.big_rest = None    # sharded: bytes after such a publish, held until it is enqueued
        self.inbuf = bytearray()
        self.out = bytearray()
        self.frame_max = 131072
        self.heartbeat = 0
        self.last_rx = self.last_tx = time.monotonic()
        self.closing_channels = set()
        self.last_queue = {}    # channel -> last declared queue name (AMQP empty-name rule)
        self.user = ""
        self.cap_blocked = False


FE_OPEN, FE_CLOSED, FE_HOST, FE_CTRL, FE_TXBUF, FE_EVENT, FE_STATUS, FE_PERSIST, FE_ERROR, FE_GROW, FE_SYNC, \
    FE_XFAIL, FE_INJECTED, FE_GET = range(1, 15)
GS_EMPTY, GS_OK, GS_RETRY, GS_NO_SPACE, GS_WINDOW_FULL, GS_GONE = range(6)   # step_abi.h GetOut.status


class _PlaneLock:
    """Exclusive access to the data plane's device tables.  With the pipelined front end
    the outermost full acquisition pauses its stepper (steps in flight finished, their
    egress written) and the release resumes it.

    ``light`` sections (``_LightLock``) share the lock but do not pause: the control work
    inside them only writes connection / channel / consumer tables, which the plane stages
    (``GpuDataPlane.defer``) for the next step's first kernel; their replies go out behind
    the egress of the steps that were in flight (``Frontend.send_after``).  A full section
    nested in a light one pauses then, and first applies what the light one staged."""

    def __init__(self, broker):
        self.b, self.rl, self.depth = broker, threading.RLock(), 0
        self.paused_at = 0   # depth of the acquisition that paused the stepper (0: running)
        self.light = 0       # open light sections

    def _defer(self, on):
        if hasattr(self.b.plane, "eng"):
            self.b.plane.defer = on

    @property
    def deferring(self):
        return self.light > 0 and not self.paused_at

    def __enter__(self):
        self.rl.acquire()
        self.depth += 1
        if not self.paused_at and self.b.fe is not None:
            self.b.stats["pauses"] = self.b.stats.get("pauses", 0) + 1
            self.b.fe.pause()
            self.paused_at = self.depth
            self._defer(False)
            if hasattr(self.b.plane, "flush_deltas"):   # what light sections staged, applied now
                self.b.plane.flush_deltas()
            if hasattr(self.b.fe, "flush_ctl"):          # and the replies held behind it written
                self.b.fe.flush_ctl()
            if hasattr(self.b.plane, "reserve_ring_chunk") and self.b.node is None:
                # rings for queues declared in light sections (no device read there)
                self.b.plane.reserve_ring_chunk(16 * self.b.plane.default_queue_capacity)
            if self.light:
                # replies a light section produced but has not queued yet: written now,
                # while paused (its staged writes were just applied; once the steps resume,
                # a consumer it activated gets deliveries, which must follow its ConsumeOk)
                self.b._flush_all()
        return self

    def __exit__(self, *exc):
        if self.paused_at == self.depth:
            self.b.fe.resume()
            self.paused_at = 0
            if self.light:
                self._defer(True)
        self.depth -= 1
        self.rl.release()


class _LightLock:
    """A control section that leaves the steps running (see ``_PlaneLock``)."""

    def __init__(self, lock):
        self.l = lock

    def _eng(self):
        return getattr(self.l.b.plane, "eng", None)

    def __enter__(self):
        lk = self.l
        lk.rl.acquire()
        lk.depth += 1
        lk.light += 1
        eng = self._eng()
        if eng is not None and hasattr(eng, "stage_begin"):
            eng.stage_begin()   # one batch per section: no step takes it before __exit__
        if not lk.paused_at:
            lk._defer(True)
            lk.b.stats["light_sections"] = lk.b.stats.get("light_sections", 0) + 1
        return self

    def __exit__(self, *exc):
        lk = self.l
        lk.light -= 1
        eng = self._eng()
        if eng is not None and hasattr(eng, "stage_end"):
            eng.stage_end()
        if not lk.light and not lk.paused_at:
            lk._defer(False)
            if lk.b.fe is not None:
                lk.b.fe.wake()   # the staged writes ride the next step
        lk.depth -= 1
        lk.rl.release()

    def cut(self):
        """Close the section's staged batch here (it rides the next step) and go on
        staging into a new one: a change set never outgrows one step's delta buffer."""
        eng = self._eng()
        if eng is not None and hasattr(eng, "stage_end"):
            eng.stage_end()
            eng.stage_begin()
            if self.l.b.fe is not None:
                self.l.b.fe.wake()


# control commands that only touch connection / channel / consumer tables: handled while
# the steps keep running (their table writes ride the next step)
_LIGHT_METHODS = {(10, 50), (10, 51), (20, 10), (20, 20), (20, 21), (20, 40), (20, 41), (30, 10), (60, 10),
                  (60, 20), (60, 30), (85, 10)}
# single node only (a sharded node replicates them through the control log): topology
# changes that only rewrite routing tables (staged whole, applied by one step's k_stage),
# and the declare of a new queue whose ring comes from the host's reserved chunk
_LIGHT_TOPOLOGY = {(40, 10), (40, 20), (50, 10), (50, 20), (50, 50)}


class _ColdStopped(Exception):
    """The broker stopped while the cold thread waited for a side operation."""


class _Hard(Exception):
    """Connection-level error: Connection.Close(code, text, class, method)."""

    def __init__(self, code, text, cls=0, mid=0):
        super().__init__(text)
        self.code, self.text, self.cls, self.mid = code, text, cls, mid


def _frames(buf):
    """Complete frames at the front of ``buf`` -> [(type, channel, payload)], consumed."""
    out, pos = [], 0
    while len(buf) - pos >= 7:
        t, ch, size = struct.unpack_from(">BHI", buf, pos)
        if len(buf) - pos < 8 + size:
            break
        if buf[pos + 7 + size] != C.FRAME_END:
            raise _Hard(C.FRAME_ERROR, "bad frame end")
        out.append((t, ch, bytes(buf[pos + 7:pos + 7 + size])))
        pos += 8 + size
    return out, pos


class GpuBroker:
    def __init__(self, plane, host="127.0.0.1", port=0, heartbeat=0, frame_max=131072, channel_max=2047,
                 idle_step_ms=2.0, product="chanamq-amd", version="0.1.0", io="native",
                 ingress_bytes=64 << 20, per_conn_read=256 << 10, mem_high_watermark=None, mem_low_watermark=None,
                 store=None, node=None, reuseport=False, io_threads=4, fe_cfg=None, spill_at=None, spill_hot=1024,
                 confirm_read=128 << 10, cold_dir=None, cold=True, cold_hot=1 << 16, cold_window=1 << 15, cold_beside=True,
                 persist_group_ms=2.0):
        """``io``: "pipeline" = native pipelined front end (csrc/core/frontend.cpp: IO
        threads + a stepper thread keeping two steps in flight, no Python per step),
        "native" = C++ batched gateway polled by a Python step loop (csrc/core/
        gateway.cpp), "python" = selectors loop (portable fallback); "auto" = pipeline
        for a single-rank GPU plane, else native."""
        self.plane = plane
        native_x = bool(getattr(plane, "native_xchg", False))
        if io == "auto":
            io = "pipeline" if (hasattr(plane, "eng") and (node is None or native_x)) else "native"
        if io == "pipeline" and (not hasattr(plane, "eng") or (node is not None and not native_x)):
            raise ValueError("io='pipeline' needs a GPU data plane (sharded: built with native_xchg=1)")
        self.io = io
        self.io_threads = io_threads
        self.fe_cfg = dict(fe_cfg or {})
        self.ctl_trace = collections.deque(maxlen=400000) if os.environ.get("CHANAMQ_CTL_TRACE") else None
        self.persist_group_ms = persist_group_ms    # extra native front-end settings (frontend.hpp FrontendCfg)
        self.gw = None
        self.fe = None
        self._fe_stats = None
        self._grow_log = []       # (front-end step count, rings moved): diagnostics
        self.ingress_bytes, self.per_conn_read = ingress_bytes, per_conn_read
        # pipelined front end: a connection with a publisher-confirm channel reads at most
        # this much per step (0 = per_conn_read).  Confirm-mode publishers hold a bounded
        # window of unconfirmed messages, so shorter steps return confirms sooner: config 4
        # over TCP at 8 IO threads 0.86 M msgs/s confirmed at 128 KiB vs 0.58 M at 512 KiB
        # (profiles/r3_e2e/config4_pcr_ab_io8.json)
        self.confirm_read = confirm_read
        # back-pressure (SURVEY A.Q17 / config 5): above the high watermark of stored
        # message bytes publishers get Connection.Blocked (if they announced the
        # capability) or Channel.Flow(active=false); released below the low watermark
        # (on by default for a GPU plane: 40% of its HBM body log; 0 = off)
        if mem_high_watermark is None:
            mem_high_watermark = int(0.4 * plane.info["log_bytes"]) if hasattr(plane, "info") else 0
        self.mem_high = mem_high_watermark
        self.mem_low = mem_low_watermark if mem_low_watermark is not None else mem_high_watermark // 2
        # the HBM message table is the other finite store: above 75% of it publishers are
        # paused too (down to 40%), else it fills before the byte watermark and drops
        msg_max = plane.info["msg_max"] if hasattr(plane, "info") else 0
        self.msg_high = int(0.75 * msg_max) if self.mem_high else 0
        self.msg_low = int(0.4 * msg_max) if self.mem_high else 0
        # and the body log's occupancy (head - tail: one old live message pins the tail):
        # publishers pause above 50% of it, resume below 25%
        log_bytes = plane.info["log_bytes"] if hasattr(plane, "info") else 0
        self.log_high = log_bytes // 2 if self.mem_high else 0
        self.log_low = log_bytes // 4 if self.mem_high else 0
        self.blocked = False
        # cold bodies to host memory (a plane built with spill_bytes): once the HBM log is
        # this full, queued messages whose bodies sit in the oldest half of the log move
        # to the host spill ring (but the first ``spill_hot`` of a queue with consumers),
        # so the log tail advances and publishers keep going until the spill ring fills
        sb = plane.info.get("spill_bytes", 0) if hasattr(plane, "info") else 0
        self.spill_at = (int(0.3 * log_bytes) if spill_at is None else int(spill_at)) if sb else 0
        self.spill_hot = spill_hot
        self._last_spill = 0.0
        # third tier (store/cold.py): once the spill ring is 60% full, spilled bodies of
        # single-queue non-persistent messages cold_hot+ entries behind their queue's head
        # go to the cold store on disk; the bodies within cold_window of a head come back
        self.cold = None
        if sb and cold:
            from ..store.cold import ColdStore
            self.cold = ColdStore(cold_dir)
            plane.cold_store = self.cold
        self.cold_hot, self.cold_window = cold_hot, cold_window
        self.cold_beside = cold_beside
        self._last_cold = self._last_cold_gc = 0.0
        self._cold_pending = False
        # durable queues x persistent messages -> store (write-behind, confirm gating)
        self.persistence = None
        self.recovered = 0
        # sharded node (parallel/node.py): every step is a lockstep collective step;
        # replicated control ops (exchanges, queues, bindings) go through the control
        # log and are answered in the step that applies them on every rank
        self.node = node
        self.reuseport = reuseport
        self._deferred = {}     # control-log seq -> (conn, channel, reply builder)
        self._rpaused = set()
        if store is not None:
            from ..engine.persistence import GpuPersistence
            self.persistence = GpuPersistence(plane, store)
            self.recovered = self.persistence.recover(int(time.time() * 1000))
        self.host, self.port = host, port
        self.heartbeat, self.frame_max, self.channel_max = heartbeat, frame_max, channel_max
        self.idle_step_s = idle_step_ms / 1000.0
        self.product, self.version = product, version
        self.conns = {}
        # slot c_max-1: pseudo-connection through which committed transactions publish
        self.txc = plane.c_max - 1
        # sharded: the slots below txc serve remote-consumer links (parallel/links.py)
        n_link = min(64, max(2, plane.c_max // 16)) if node is not None else 0
        self._top_slot = plane.c_max - 2 - n_link          # highest client connection slot
        self._free = list(range(self._top_slot, 0, -1))   # slot 0 unused
        self._link_free = list(range(self._top_slot + 1, plane.c_max - 1))
        self._links = {}        # (conn, channel, consumer tag) -> link id (remote consumers)
        self._get_links = {}    # (vhost, queue) -> get link id (Basic.Get of remote queues)
        self._get_wait = {}     # pull id -> (conn, channel, no_ack, link id)
        self._dev_gets = {}     # Basic.Gets queued on the device: id -> (conn, channel, queue slot, no_ack, vhost,
        #                         queue, resume: the answer unpauses the connection)
        self._dget_ctx = False  # handling a step-decoded Basic.Get (its connection is not paused)
        self._get_holders = {}  # get link id -> {(conn, channel)} holding unacked Get messages
        self._get_used = {}     # get link id -> monotonic time of its last Get
        self._pull_seq = 0
        self._link_seq = 0
        if node is not None:
            node.links._alloc = self._alloc_link_slot
            node.links._free = self._link_free.append
        self._txbuf = {}        # (conn, channel) -> raw data commands held since Tx.Select / last commit
        self._tx_pending = []   # commits waiting for their injection step: (conn, channel, bytes)
        self._tx_active = None  # (conn, channel) injected in the current step
        self._sel = selectors.DefaultSelector()
        self._lsock = None
        self._thread = None
        self._running = False
        self._wake_r, self._wake_w = os.pipe()
        self.stats = dict(steps=0, published=0, delivered=0, connections=0)
        self.lock = _PlaneLock(self)
        self.light = _LightLock(self.lock)

    # ------------------------------------------------------------------ lifecycle
    _live = None   # started, not yet stopped (tests stop what a failed test left running)

    def start(self):
        import weakref
        if GpuBroker._live is None:
            GpuBroker._live = weakref.WeakSet()
        GpuBroker._live.add(self)
        if self.io == "pipeline":
            from ..broker import load
            if hasattr(self.plane, "reserve_ring_chunk") and self.node is None:
                self.plane.reserve_ring_chunk(16 * self.plane.default_queue_capacity)
            self.fe = load().Frontend(self.plane.eng.c_api(), dict(
                host=self.host, port=self.port, io_threads=self.io_threads, per_conn_read=self.per_conn_read,
                idle_step_ms=self.idle_step_s * 1000.0, worker=self.plane.worker, max_slot=self._top_slot,
                reuseport=self.reuseport, **self.fe_cfg))
            self.port = self.fe.port
            if self.persistence is not None:   # native write-behind: records never touch Python
                self._pw = load().PersistWorker(self.persistence.store)
                if self.persist_group_ms > 0:   # see PersistWorker::set_group_delay
                    self._pw.set_group_delay(float(self.persist_group_ms))
                self.fe.attach_persist(self._pw)
                self.persistence.attach_native(self._pw)
            if self.node is not None:
                # sharded: lockstep steps with the native exchange; control-log syncs and
                # failovers happen at FE_SYNC / FE_XFAIL; the failure detector's heartbeat
                # is gated on this rank's step progress; remote consumers ride the device
                # exchange (DeviceLinks) when the engine has links
                self.node.attach_frontend(self.fe)
                if self.plane.info.get("links"):
                    self.node.use_device_links(self._alloc_link_slot, self._link_free.append)
                self.node.log.handlers["big_publish"] = self._apply_big
                if self.persistence is not None:
                    self.node.log.on_applied = self._persist_replicated
            self._running = True
            self.fe.start()
            self._thread = threading.Thread(target=self._loop_pipeline, name="gpu-broker-ctl", daemon=True)
            self._thread.start()
            if self._cold_beside():
                self._cold_thread = threading.Thread(target=self._cold_loop, name="gpu-broker-cold", daemon=True)
                self._cold_thread.start()
            return self
        if self.io == "native":
            from ..broker import load
            self.gw = load().Gateway(self.host, self.port, self._top_slot + 1, self.reuseport)
            self.port = self.gw.port
            if hasattr(self.plane, "mod"):
                self._pin = self.plane.mod.alloc_pinned(self.ingress_bytes)
            else:
                import numpy as np
                self._pin = np.zeros(self.ingress_bytes, np.uint8)
            self._running = True
            self._thread = threading.Thread(target=self._loop_native, name="gpu-broker", daemon=True)
            self._thread.start()
            return self
        ls = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        ls.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        ls.bind((self.host, self.port))
        ls.listen(1024)
        ls.setblocking(False)
        self.port = ls.getsockname()[1]
        self._lsock = ls
        self._sel.register(ls, selectors.EVENT_READ, "listen")
        self._sel.register(self._wake_r, selectors.EVENT_READ, "wake")
        self._running = True
        self._thread = threading.Thread(target=self._loop, name="gpu-broker", daemon=True)
        self._thread.start()
        return self

    def stop(self):
        if GpuBroker._live is not None:
            GpuBroker._live.discard(self)
        self._running = False
        os.write(self._wake_w, b"x")
        if self._thread:
            self._thread.join(timeout=10)
        if getattr(self, "_cold_thread", None) is not None:
            self._cold_thread.join(timeout=10)
        if getattr(self, "_pw", None) is not None:
            # shutdown is not a client close: what the open connections hold unacked stays in
            # queue_unacks (redelivered first on restart), so the requeue records the drops
            # below produce on the still-running stepper are not committed
            self._pw.drain()
            self._pw.stop()
        for c in list(self.conns.values()):
            self._drop(c)
        if self.fe is not None:
            self.fe.stop()
            self._sync_fe_stats()
            if getattr(self, "_pw", None) is not None:
                self._pw.stop()
                self._pw_stats = self._pw.stats()
            self.fe = None
        self._sel.close()
        if self._lsock is not None:
            self._lsock.close()
        self.gw = None
        if self.cold is not None:
            self.cold.close()
        os.close(self._wake_r)
        os.close(self._wake_w)

    # ------------------------------------------------------------------ admin (server/admin.py)
    def create_vhost(self, name):
        with self.lock:
            self.plane.ensure_vhost(name)
            if self.persistence is not None:
                self.persistence.vhost(name)
                self.persistence.control_commit()
        return True

    def delete_vhost(self, name):
        # reference parity (A.Q28): no cascade; the vhost stays usable by open connections
        return True

    def stats_json(self):
        import json
        with self.lock:
            d = dict(self.stats)
            d.update(connections_open=sum(1 for c in self.conns.values() if c.state == "open"),
                     queues=len(self.plane.queues), exchanges=len(self.plane.exchanges),
                     stored_bytes=self.plane.memory_in_use(), blocked=self.blocked)
        return json.dumps(d)

    def queues_json(self):
        import json
        with self.lock:
            out = [{"vhost": q.vhost, "name": q.name, "durable": q.durable, "owner": q.owner,
                    "ready": self.plane.message_count(q.slot) if q.owner == self.plane.rank else None,
                    "consumers": len(q.consumers)} for q in self.plane.queues.values()]
        return json.dumps(out)

    # ------------------------------------------------------------------ pipelined native loop
    def _loop_pipeline(self):
        """Control plane of the native front end: blocks on its events (handshakes,
        control commands, closes, store records) and takes the device (``self.lock``
        pauses the stepper) only while it handles them; steps never wait for Python."""
        fe = self.fe
        last_stats = 0.0
        # with body tiers the movers must keep pace with the publishers (a full HBM log and
        # spill ring would nack): 5 ms upkeep instead of 50
        tiers = bool(self.spill_at) or self.cold is not None
        period = 0.005 if tiers else 0.05
        while self._running:
            evs = fe.poll_events(5 if tiers else 20)
            persist = [e for e in evs if e[0] == FE_PERSIST]
            dev = self._fast_events([e for e in evs if e[0] != FE_PERSIST])
            if dev or self._tx_pending:
                light = not self._tx_pending and self._light_ok(dev)
                with (self.light if light else self.lock):
                    while dev or (self._tx_pending and self.node is None):
                        if light and not self._light_ok(dev):
                            with self.lock:   # a command that needs the device drained
                                self._handle_fe(dev)
                        elif light:
                            # a few commands at a time: once the staged set nears what one
                            # step applies, the batch is cut there (each command's writes stay
                            # in one step's batch: ADVICE r5)
                            for k in range(0, len(dev), 16):
                                n, nb, _ = self.plane.deltas_pending()
                                if k and (n > 256 or nb > (1 << 20)):
                                    self.light.cut()
                                self._handle_fe(dev[k:k + 16])
                        else:
                            self._handle_fe(dev)
                        if self.node is not None:   # sharded: injected into the lockstep steps
                            self._tx_inject()
                        while self._tx_pending and self.node is None:   # committed transactions:
                            self._host_step({})                         # host-run injection steps
                        more = fe.poll_events(0)
                        persist += [e for e in more if e[0] == FE_PERSIST]
                        dev = [e for e in more if e[0] != FE_PERSIST]
                    if self.persistence is not None and self.plane._get_consumed:
                        self._persist_gets()
                    self._flush_all()
            if persist:
                self._persist_native(persist)
            now = time.monotonic()
            if now - last_stats > period:
                last_stats = now
                self._sync_fe_stats()
                self._watermarks()
                self._flush_all()

    # ------------------------------------------------------------------ light control sections
    def _light_capable(self):
        # (a store is no obstacle: the light commands write no store rows -- consumer sets are
        # not persisted -- and their replies wait only for the held steps carrying bytes of
        # their own connection, Frontend::release_ctl)
        return (self.fe is not None and hasattr(self.plane, "eng") and hasattr(self.fe, "send_after")
                and (self.node is None or getattr(self.plane, "native_xchg", False)))

    def _close_light(self, c):
        """A connection whose close only releases connection / channel / consumer rows --
        and, on a single node, its exclusive queues (deleted without device reads,
        GpuDataPlane.queue_deleted) -- with no remote-consumer link to close through the
        control log."""
        if any(k[0] == c.id for k in self._links):
            return False
        return self.node is None or not any(q.exclusive_owner == c.id for q in self.plane.queues.values())

    def _topology_light(self, c, key, data):
        """Exchange / queue / binding commands handled beside the steps (single node)."""
        if self.node is not None or key not in _LIGHT_TOPOLOGY:
            return False
        if key != (50, 10):
            return True
        try:
            m = decode_method(bytes(data[7:]))
        except Exception:   # noqa: BLE001 - malformed: the full path reports it
            return False
        pc = self.plane.conns.get(c.id)
        if m.passive or pc is None or (m.queue and (pc.vhost, m.queue) in self.plane.queues):
            return False   # (an existing queue's DeclareOk needs its message count: a device read)
        cap = 1
        while cap < self.plane.default_queue_capacity:
            cap <<= 1
        return hasattr(self.plane, "ring_light_ok") and self.plane.ring_light_ok(cap)

    def _consume_light(self, c, data):
        """Basic.Consume / Cancel in a light section: on a sharded node only for a queue this
        rank owns (a remote queue is a link through the control log) / a local consumer."""
        if self.node is None:
            return True
        try:
            m = decode_method(bytes(data[7:]))
        except Exception:   # noqa: BLE001 - malformed: the full path reports it
            return False
        ch = struct.unpack_from(">H", data, 1)[0]
        if m.name == "basic.cancel":
            return (c.id, ch, m.consumer_tag) not in self._links
        pc = self.plane.conns.get(c.id)
        q = self.plane.queues.get((pc.vhost if pc else "", m.queue or c.last_queue.get(ch, "")))
        return q is not None and q.owner == self.plane.rank

    def _plock(self):
        """The lock for a light-safe operation: light inside a light section, else full."""
        return self.light if self.lock.deferring else self.lock

    def _light_ok(self, evs):
        """Whether this batch of front-end events can be handled with the steps running:
        handshakes, channel / consumer / QoS / confirm commands and plain closes; anything
        that reads device state or changes queues, exchanges or bindings needs the drain."""
        why = self._light_why(evs)
        if why is not None:   # (why the stepper pauses: stats["pause_why"], by cause)
            pw = self.stats.setdefault("pause_why", {})
            pw[why] = pw.get(why, 0) + 1
        return why is None

    def _light_why(self, evs):
        if not self._light_capable():
            return "not light-capable"
        n, nb, nd = self.plane.deltas_pending()
        if n > 256 or nb > (1 << 20) or nd > 1024:   # a change set must fit one step's delta buffer
            return "staged writes"
        for kind, conn, a, b, data, data2 in evs:
            if kind in (FE_OPEN, FE_GET, FE_EVENT, FE_STATUS, FE_TXBUF):
                continue
            c = self.conns.get(conn)
            if kind == FE_CLOSED:
                if c is not None and c.state == "open" and not self._close_light(c):
                    return "close with exclusive queues"
            elif kind == FE_HOST:
                # handshakes and the close handshake; on an open connection a stale event (its
                # bytes went to the data plane with set_data_mode) -- nothing reads the device
                if c is not None and (c.state not in ("header", "start", "tune", "closing", "open") or c.big is not None):
                    return "host bytes " + c.state
            elif kind == FE_CTRL:
                if c is None or c.state != "open" or len(data) < 11:
                    continue
                ch = struct.unpack_from(">H", data, 1)[0]
                if ch in c.closing_channels:
                    continue
                key = struct.unpack_from(">HH", data, 7)
                if data[0] == C.FRAME_METHOD and key in _LIGHT_TOPOLOGY and self._topology_light(c, key, data):
                    continue
                if data[0] != C.FRAME_METHOD or key not in _LIGHT_METHODS:
                    return "method %d.%d" % key if data[0] == C.FRAME_METHOD else "content"
                if key == (10, 50) and not self._close_light(c):
                    return "close with exclusive queues"
                if key == (20, 40) and any(k[0] == c.id and k[1] == ch for k in self._links):
                    return "channel close with remote consumers"
                if key in ((60, 20), (60, 30)) and not self._consume_light(c, data):
                    return "remote consumer"
            else:
                return "event %d" % kind
        return None

    def _fast_events(self, dev):
        """Basic.Get traffic without pausing the stepper: a Get on a local queue is staged
        for the next step (fe.queue_get) and its answer (FE_GET) replied to right away --
        neither touches device state (the getting connection's unpause rides the next
        step, GpuDataPlane.unpause).  Returns the events left for the locked path."""
        if self.node is not None or not hasattr(self.plane, "eng"):
            return dev
        rest = []
        for e in dev:
            kind, conn = e[0], e[1]
            if kind == FE_GET and (e[2] & 0xFFFFFFFF) in (GS_OK, GS_EMPTY, GS_RETRY, GS_GONE):
                self._get_answer(conn, e[2], e[3])
                continue
            if kind == FE_CTRL and self._fast_get(conn, e[4], resume=e[2] != 1):
                continue
            rest.append(e)
        return rest

    def _fast_get(self, conn, raw, resume=True):
        c = self.conns.get(conn)
        if c is None or c.state != "open" or len(raw) < 11:
            return False
        t, ch, size = struct.unpack_from(">BHI", raw, 0)
        if t != C.FRAME_METHOD or struct.unpack_from(">HH", raw, 7) != (60, 70) or ch in c.closing_channels:
            return False
        p = self.plane
        pc = p.conns.get(c.id)
        if pc is None or ch not in pc.channels:
            return False
        m = decode_method(bytes(raw[7:7 + size]))
        q = p.queues.get((pc.vhost, m.queue or c.last_queue.get(ch, "")))
        if q is None or q.exclusive_owner not in (-1, c.id) or q.owner != p.rank:
            return False   # errors and remote queues: the locked path
        gid = self._next_get = getattr(self, "_next_get", 0) + 1
        self._dev_gets[gid] = (c.id, ch, q.slot, bool(m.no_ack), pc.vhost, q.name, resume)
        self.fe.queue_get(c.id, p.chslot(c.id, ch), q.slot, int(bool(m.no_ack)), gid)
        self.stats["device_gets"] = self.stats.get("device_gets", 0) + 1
        return True

    def _handle_fe(self, evs):
        ctrl, events, seg_status, txbuf = [], [], [], []
        sync = None
        for kind, conn, a, b, data, data2 in evs:
            if kind in (FE_SYNC, FE_XFAIL):
                sync = kind if sync is None else max(sync, kind)
                continue
            if kind == FE_INJECTED:   # a committed transaction's publishes were stepped
                if conn == self.txc:
                    self._tx_end()
                continue
            if kind == FE_GET:        # a Basic.Get answered by its step
                self._get_answer(conn, a, b)
                continue
            if kind == FE_OPEN:
                self.conns[conn] = _Conn(None, conn, None)
                self.stats["connections"] += 1
            elif kind == FE_CLOSED:
                c = self.conns.get(conn)
                if c is not None:
                    c.state = "gone"
                    self._drop(c)
                else:   # (a: the slot's generation -- it may have been freed and reused since)
                    self.fe.close(conn, a)
            elif kind == FE_HOST:
                c = self.conns.get(conn)
                data = self.fe.take(conn)
                if c is None or not data:
                    continue
                was_open = c.state == "open"
                rest = self._host_bytes(c, data)
                if c.state == "open" and not was_open:
                    self._flush(c, direct=True)   # Connection.OpenOk: no device traffic yet
                    self.fe.set_heartbeat(conn, c.heartbeat)
                    self.fe.set_data_mode(conn, rest)
            elif kind == FE_CTRL:   # (a == 1: a Basic.Get its step decoded but could not serve)
                ctrl.append((conn, data, a == 1))
            elif kind == FE_TXBUF:
                txbuf.append((conn, a, data))
            elif kind == FE_EVENT:
                events.append((conn, a, b))
            elif kind == FE_STATUS:
                seg_status.append((conn, a))
            elif kind == FE_GROW:   # the device grew rings: return the old ranges to the pool
                self.plane.rings_moved(data)
                if len(self._grow_log) < 256:
                    self._grow_log.append(((self._fe_stats or {}).get("steps", 0), len(data) // 56))
            elif kind == FE_ERROR:
                import logging
                logging.getLogger("chanamq.gpu").error("data-plane engine failed: %s", data.decode(errors="replace"))
                self._running = False
        if ctrl or events or seg_status or txbuf:
            txbuf.sort()
            self._after_step(ctrl, events, seg_status, {}, False, False, txbuf)
        if sync is not None:
            self._sync_point(sync == FE_XFAIL)

    def _sync_point(self, failed):
        """Every rank's stepper parked at the same step (no exchange in flight): fail over
        if a peer stopped answering, then apply the replicated control log everywhere and
        answer this rank's deferred control commands; the steps resume afterwards."""
        node = self.node
        try:
            if failed:
                node.failover_point()
            self._answer(node.sync_point())
            if self._get_wait or self._get_links:   # remote Basic.Get answers restored at this sync
                self._serve_gets()
            if self.persistence is not None:
                self.persistence.control_commit()
        finally:
            self.fe.sync_done()

    def _persist_replicated(self, op, args, kw, res):
        """Durable topology applied from the control log goes into this rank's store too
        (every rank holds the replicated exchanges / queues / bindings; a survivor adopting
        a dead rank's queues finds their rows)."""
        from ..parallel.control_log import error_of
        if error_of(res) or self.persistence is None:
            return
        p, ps = self.plane, self.persistence
        if op == "declare_exchange":
            x = p.exchanges.get((args[0], args[1]))
            if x is not None:
                ps.exchange(x)
        elif op == "delete_exchange":
            ps.exchange_deleted(args[0], args[1])
        elif op == "declare_queue":
            q = p.queues.get((args[0], args[1]))
            if q is not None:
                ps.queue(q)
        elif op == "delete_queue":
            ps.queue_deleted(args[0], args[1])
        elif op == "bind":
            ps.bind(*args[:4])
        elif op == "unbind":
            ps.unbind(*args[:4])

    def _persist_native(self, evs):
        """Write-behind group commit: the store rows of every held step in this batch,
        one fsync, then their egress (with the publisher confirms) is released."""
        from ..engine.dataplane import parse_consumed, parse_persist
        top = max(e[2] for e in evs)
        if self.persistence is not None:
            for kind, conn, step, overflow, data, data2 in evs:
                if overflow:
                    raise RuntimeError("persist buffer overflow: raise persist_max / persist_bytes")
                self.persistence.apply(parse_persist(data) if data else [], parse_consumed(data2) if data2 else [])
            self.persistence.commit()
        self.fe.release(top)

    def _persist_gets(self):
        """Store records of Basic.Get calls (between steps, no step collected them)."""
        if self.persistence.native is not None:
            from ..engine.layout import CONSUMED_REC
            gets = self.plane.take_get_consumed()
            a = np.zeros(len(gets), CONSUMED_REC)
            for i, (mid, q, qpos, kind) in enumerate(gets):
                a[i] = (mid, qpos, q, kind, (0, 0))
            self.persistence.submit_raw(b"", a.tobytes())
        else:
            self.persistence.apply([], self.plane.take_get_consumed())
            self.persistence.commit()

    def _sync_fe_stats(self):
        if self.fe is None:
            return
        st = self.fe.stats()
        self.stats.update(steps=st["steps"], published=st["published"], delivered=st["delivered"])
        if st.get("spill_moved"):
            self.stats["spilled_bytes"] = st["spill_moved"]
        self._fe_stats = st
        pw = getattr(self, "_pw", None)
        if pw is not None and "store_failed" not in self.stats:
            ps = pw.stats()
            if ps["failed"]:   # held confirms -> Nack, publishers blocked; fe.healthy() False (sharded: fail over)
                self.stats["store_failed"] = ps["error"]
                import logging
                logging.getLogger("chanamq.gpu").error("persistent store failed: unconfirmed publishes are nacked, "
                                                       "publishers blocked: %s", ps["error"])
                self._watermarks()
        if st.get("store_fail_nacks"):
            self.stats["store_fail_nacks"] = st["store_fail_nacks"]

    def _host_step(self, inputs):
        """A synchronous step run by the control plane while the front end is paused
        (transaction injection, queue purge): only the given connections take part; its
        egress goes out through the front end."""
        inj = self._tx_begin()
        if inj:
            inputs = dict(inputs)
            inputs[self.txc] = inj
        res = self.plane.step(inputs, now_ms=int(time.time() * 1000), with_carry=False)
        self._persist_step()
        egress = dict(res.egress)
        if self.txc in egress:
            data = egress.pop(self.txc)
            if self._tx_active is not None:
                egress[self._tx_active[0]] = egress.get(self._tx_active[0], b"") + data
        for conn, data in egress.items():
            c = self.conns.get(conn)
            if c is not None and c.state == "open":
                c.out += data
        seg_status = [(sg[0], sg[1]) for sg in res.segs]
        self._after_step(res.ctrl, res.events, seg_status, res.counters, bool(inputs), bool(egress), res.txbuf)

    # ------------------------------------------------------------------ native loop
    def _loop_native(self):
        import numpy as np

        from ..engine.layout import SEG_IN
        gw, pin = self.gw, self._pin
        gpu = hasattr(self.plane, "eng")
        last_step = 0.0
        busy = False
        while self._running:
            timeout_ms = 0 if busy else max(1, int(self.idle_step_s * 1000))
            segs_b, used, hs, opened, closed = gw.poll(timeout_ms, pin, 0, self.per_conn_read)
            now = time.monotonic()
            for cid in opened:
                self.conns[cid] = _Conn(None, cid, None)
                self.stats["connections"] += 1
            for cid in closed:
                c = self.conns.get(cid)
                if c is not None:
                    c.state = "gone"
                    self._drop(c)
            segs = np.frombuffer(segs_b, SEG_IN).copy()
            extra = []
            for cid, data in hs:
                c = self.conns.get(cid)
                if c is None:
                    continue
                c.last_rx = now
                rest = self._host_bytes(c, data)
                if c.state == "open":
                    gw.set_data_mode(cid, True)
                if rest:
                    extra.append((cid, rest))
            for cid in segs["conn"]:
                c = self.conns.get(int(cid))
                if c is not None:
                    c.last_rx = now
            if extra:
                rows = []
                for cid, data in extra:
                    off = (used + 15) & ~15
                    pin[off:off + len(data)] = np.frombuffer(data, np.uint8)
                    rows.append((cid, len(data), off))
                    used = off + len(data)
                segs = np.concatenate([segs, np.array(rows, SEG_IN)])
            if gpu:
                have = set(int(x) for x in segs["conn"])
                add = [(int(cc), 0, 0) for cc in np.nonzero(self.plane.carry)[0]
                       if int(cc) not in have and int(cc) in self.plane.conns and not self.plane.conns[int(cc)].paused]
                if add:
                    segs = np.concatenate([segs, np.array(add, SEG_IN)])
            open_conns = any(c.state == "open" for c in self.conns.values())
            if self.node is not None:     # lockstep: every rank steps every tick
                with self.lock:
                    busy = self._step_native(segs, used, gpu)
                last_step = now
            elif open_conns and (len(segs) or busy or now - last_step >= self.idle_step_s):
                with self.lock:
                    busy = self._step_native(segs, used, gpu)
                last_step = now
            else:
                busy = False
            self._heartbeats(now)
            self._flush_all()
            gw.flush()

    def _step_native(self, segs, used, gpu):
        if not gpu:   # golden plane: bytes per connection
            inputs = {int(r["conn"]): bytes(self._pin[int(r["src"]):int(r["src"]) + int(r["len"])]) for r in segs}
            return self._step(inputs)
        p = self.plane
        now = int(time.time() * 1000)
        inj = self._tx_begin()
        if inj:
            off = (used + 15) & ~15
            self._pin[off:off + len(inj)] = np.frombuffer(inj, np.uint8)
            segs = np.concatenate([segs, np.array([(self.txc, len(inj), off)], segs.dtype)])
            used = off + len(inj)
        if self.node is not None:
            if self._get_wait or self._get_links:
                self._serve_gets()
            t, results = self.node.step_raw(segs, self._pin.ctypes.data, used, now)
            self._answer(results)
        else:
            t = p.submit_raw(segs, self._pin.ctypes.data, used, now)
        res = p.finish(t, collect=True, collect_egress=False)
        self._persist_step()
        eg, co = p.host_egress(t)
        if self.node is not None and self.node.links.active:   # remote consumers: link traffic
            pe = {}
            for lk in self.node.links.links.values():
                if lk.pc is not None and co["len"][lk.pc]:
                    o, n = int(co["off"][lk.pc]), int(co["len"][lk.pc])
                    pe[lk.pc] = bytes(eg[o:o + n])
                    co["len"][lk.pc] = 0
            self.node.relay(pe)
        if co["len"][self.txc]:    # Basic.Return of committed publishes -> their connection
            o, n = int(co["off"][self.txc]), int(co["len"][self.txc])
            if self._tx_active is not None and self._tx_active[0] in self.conns:
                self.gw.send(self._tx_active[0], bytes(eg[o:o + n]))
            co["len"][self.txc] = 0
        self.gw.send_egress(eg, co.view(np.uint32), p.c_max)
        self._read_backpressure(segs)
        return self._after_step(res.ctrl, res.events, [(s[0], s[1]) for s in res.segs], res.counters,
                                bool(len(segs)), bool(co["len"].any()), res.txbuf)

    # ------------------------------------------------------------------ loop
    def _loop(self):
        last_step = 0.0
        busy = False
        while self._running:
            timeout = 0 if busy else self.idle_step_s
            inputs = {}
            for key, _ in self._sel.select(timeout):
                if key.data == "listen":
                    self._accept()
                elif key.data == "wake":
                    os.read(self._wake_r, 64)
                else:
                    self._read(key.data, inputs)
            now = time.monotonic()
            open_conns = any(c.state == "open" for c in self.conns.values())
            if open_conns and (inputs or busy or now - last_step >= self.idle_step_s):
                with self.lock:
                    busy = self._step(inputs)
                last_step = now
            else:
                busy = False
            self._heartbeats(now)
            self._flush_all()

    def _accept(self):
        try:
            s, peer = self._lsock.accept()
        except BlockingIOError:
            return
        if not self._free:
            s.close()
            return
        s.setblocking(False)
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        c = _Conn(s, self._free.pop(), peer)
        self.conns[c.id] = c
        self._sel.register(s, selectors.EVENT_READ, c)
        self.stats["connections"] += 1

    def _read(self, c, inputs):
        try:
            data = c.sock.recv(1 << 18)
        except (BlockingIOError, InterruptedError):
            return
        except OSError:
            data = b""
        if not data:
            self._drop(c)
            return
        c.last_rx = time.monotonic()
        if c.state == "open":
            inputs[c.id] = inputs.get(c.id, b"") + data
            return
        rest = self._host_bytes(c, data)
        if rest:
            inputs[c.id] = rest

    def _host_bytes(self, c, data):
        """Bytes of a connection that is not (yet / any more) on the data plane:
        handshake, a large publish being assembled, or waiting for Connection.CloseOk.
        Returns data-plane leftovers."""
        if c.state == "bigpub":
            return self._big_feed(c, data)
        if c.state == "bigwait":   # held until the sharded large publish is enqueued
            c.big_rest += data
            return b""
        if c.state in ("header", "start", "tune"):
            c.inbuf += data
            try:
                return self._handshake(c)
            except _Hard as e:
                self._conn_close(c, e.code, e.text, e.cls, e.mid)
            except ControlError as e:
                self._conn_close(c, e.code, e.text, e.class_id, e.method_id)
            return b""
        if c.state == "closing":
            c.inbuf += data
            frames, used = _frames(c.inbuf)
            del c.inbuf[:used]
            for t, ch, payload in frames:
                if t == C.FRAME_METHOD and ch == 0:
                    m = decode_method(payload)
                    if m.name in ("connection.close_ok", "connection.close"):
                        if m.name == "connection.close":
                            self._send(c, 0, Method("connection.close_ok"))
                        self._flush(c)
                        self._drop(c)
                        return b""
        return b""

    # ------------------------------------------------------------------ handshake (host)
    def _handshake(self, c):
        if c.state == "header":
            if len(c.inbuf) < 8:
                return b""
            if bytes(c.inbuf[:8]) != C.PROTOCOL_HEADER:
                c.out += C.PROTOCOL_HEADER
                self._flush(c)
                self._drop(c)
                return b""
            del c.inbuf[:8]
            caps = {"publisher_confirms": True, "exchange_exchange_bindings": False, "basic.nack": True,
                    "consumer_cancel_notify": True, "connection.blocked": False}
            self._send(c, 0, Method("connection.start", version_major=0, version_minor=9,
                                    server_properties={"product": self.product, "version": self.version,
                                                       "capabilities": caps},
                                    mechanisms=b"PLAIN AMQPLAIN EXTERNAL", locales=b"en_US"))
            c.state = "start"
        frames, used = _frames(c.inbuf)
        consumed = 0
        for k, (t, ch, payload) in enumerate(frames):
            if t == C.FRAME_HEARTBEAT:
                continue
            if t != C.FRAME_METHOD or ch != 0:
                raise _Hard(C.UNEXPECTED_FRAME, "unexpected frame during handshake")
            m = decode_method(payload)
            if m.name == "connection.start_ok" and c.state == "start":
                caps = (m.client_properties or {}).get("capabilities") or {}
                c.cap_blocked = bool(caps.get("connection.blocked", False)) if isinstance(caps, dict) else False
                mech = m.mechanism
                if mech not in ("PLAIN", "AMQPLAIN", "EXTERNAL"):
                    raise _Hard(C.ACCESS_REFUSED, f"unsupported SASL mechanism {mech}", 10, 11)
                if mech == "PLAIN":
                    parts = bytes(m.response).split(b"\0")
                    c.user = parts[1].decode("utf-8", "replace") if len(parts) > 1 else ""
                self._send(c, 0, Method("connection.tune", channel_max=self.channel_max,
                                        frame_max=self.frame_max, heartbeat=self.heartbeat))
                c.state = "tune"
            elif m.name == "connection.tune_ok" and c.state == "tune":
                fm = m.frame_max or self.frame_max
                if fm > self.frame_max or fm < 4096:
                    raise _Hard(C.SYNTAX_ERROR, f"frame-max {fm} outside negotiated range", 10, 31)
                c.frame_max = fm
                c.heartbeat = m.heartbeat
            elif m.name == "connection.open" and c.state == "tune":
                vh = normalize_vhost(m.virtual_host)
                if vh not in self.plane.vhosts:
                    raise _Hard(C.NOT_FOUND, f"no vhost '{vh}'", 10, 40)
                with self._plock():
                    self.plane.open_connection(c.id, vh, c.frame_max)
                self._send(c, 0, Method("connection.open_ok"))
                c.state = "open"
                # bytes after Connection.Open belong to the data plane
                rest = bytes(c.inbuf[self._frame_end(c.inbuf, k)[0]:])
                c.inbuf.clear()
                return rest
            else:
                raise _Hard(C.COMMAND_INVALID, f"unexpected {m.name} during handshake", m.class_id, m.method_id)
            consumed = used
        del c.inbuf[:used]
        return b""

    @staticmethod
    def _frame_end(buf, k):
        pos = 0
        for _ in range(k + 1):
            size = struct.unpack_from(">I", buf, pos + 3)[0]
            pos += 8 + size
        return pos, None

    # ------------------------------------------------------------------ data-plane step
    def _step(self, inputs):
        inj = self._tx_begin()
        if inj:
            inputs = dict(inputs)
            inputs[self.txc] = inj
        if self.node is not None:
            if self._get_wait or self._get_links:
                self._serve_gets()
            res, results = self.node.step(inputs, now_ms=int(time.time() * 1000))
            self._answer(results)
        else:
            res = self.plane.step(inputs, now_ms=int(time.time() * 1000))
        self._persist_step()
        if isinstance(res, dict):   # golden plane
            egress, ctrl, events, segs, cnt = res["egress"], res["ctrl"], res["events"], res["segs"], \
                res.get("counters", {})
            seg_status = [(s[0], s[1]) for s in segs]
            txbuf = res.get("txbuf", [])
        else:
            egress, ctrl, events, cnt = res.egress, res.ctrl, res.events, res.counters
            seg_status = [(s[0], s[1]) for s in res.segs]
            txbuf = res.txbuf
        egress = dict(egress)
        if self.txc in egress:     # Basic.Return of committed publishes -> their connection
            data = egress.pop(self.txc)
            if self._tx_active is not None:
                egress[self._tx_active[0]] = egress.get(self._tx_active[0], b"") + data
        for conn, data in egress.items():
            c = self.conns.get(conn)
            if c is not None and c.state == "open":
                if self.gw is not None:
                    self.gw.send(conn, data)
                else:
                    c.out += data
        return self._after_step(ctrl, events, seg_status, cnt, bool(inputs), bool(egress), txbuf)

    # ------------------------------------------------------------------ transactions
    def _tx_begin(self):
        """Bytes of the next committed transaction's publishes, injected this step through
        the pseudo-connection ``txc`` (same vhost, channel number and frame-max as the
        committing connection); its Tx.CommitOk goes out after the step."""
        self._tx_active = None
        while self._tx_pending:
            conn, ch, data = self._tx_pending.pop(0)
            c = self.conns.get(conn)
            pc = self.plane.conns.get(conn)
            if c is None or pc is None or c.state != "open":
                continue
            with self.lock:
                self.plane.close_connection(self.txc)
                self.plane.open_connection(self.txc, pc.vhost, pc.frame_max)
                self.plane.open_channel(self.txc, ch)
            self._tx_active = (conn, ch)
            return data
        return b""

    def _tx_inject(self):
        """Sharded pipelined node: the next committed transaction's publishes go through
        the pseudo-connection ``txc`` in the next lockstep step (a host-run step would
        bypass the exchange); Tx.CommitOk and the unpause follow at FE_INJECTED."""
        if self._tx_active is not None or not self._tx_pending:
            return
        data = self._tx_begin()
        if data:
            self.fe.inject(self.txc, data)

    def _tx_end(self):
        """After the injection step: Tx.CommitOk, and the connection resumes."""
        if self._tx_active is None:
            return
        conn, ch = self._tx_active
        self._tx_active = None
        c = self.conns.get(conn)
        if c is not None and c.state == "open":
            self._send(c, ch, Method("tx.commit_ok"))
            self._unpause(conn)
        if self.node is not None and self.fe is not None:
            self._tx_inject()

    def _tx_commit(self, c, ch):
        """Apply the channel's held acks now (window marks between steps) and queue its
        publishes for injection; returns "deferred" when CommitOk waits for that step."""
        held = self._txbuf.get((c.id, ch), [])
        self._txbuf[(c.id, ch)] = []
        pubs = []
        for raw in held:
            t, _, size = struct.unpack_from(">BHI", raw, 0)
            cls, mid = struct.unpack_from(">HH", raw, 7)
            if (cls, mid) == (60, 40):
                pubs.append(raw)
                continue
            m = decode_method(raw[7:7 + size])
            if m.name == "basic.ack":
                self.plane.apply_ack(c.id, ch, m.delivery_tag, m.multiple, False, "ack")
            elif m.name == "basic.nack":
                self.plane.apply_ack(c.id, ch, m.delivery_tag, m.multiple, m.requeue, "nack")
            elif m.name == "basic.reject":
                self.plane.apply_ack(c.id, ch, m.delivery_tag, False, m.requeue, "reject")
        if not pubs:
            self._send(c, ch, Method("tx.commit_ok"))
            return None
        self._tx_pending.append((c.id, ch, b"".join(pubs)))
        return "deferred"

    def _after_step(self, ctrl, events, seg_status, cnt, had_input, had_egress, txbuf=()):
        if self.node is None or self.fe is None:   # sharded pipelined: at FE_INJECTED
            self._tx_end()
        for conn, _, raw in txbuf:   # data commands of transactional channels, in wire order
            ch = struct.unpack_from(">H", raw, 1)[0]
            if (conn, ch) in self._txbuf:
                self._txbuf[(conn, ch)].append(raw)
        if not self.lock.deferring:   # (tier upkeep reads the device: outside light sections)
            self._watermarks()
        self.stats["steps"] += 1
        self.stats["published"] += cnt.get("n_pubs", 0)
        self.stats["delivered"] += cnt.get("n_deliv", 0)
        for conn, code, chslot in events:
            c = self.conns.get(conn)
            if c is None or c.state != "open":
                continue
            if code == C.RESOURCE_ERROR:   # the step's control buffer overflowed: command lost
                self._conn_close(c, C.RESOURCE_ERROR, "control command buffer full")
                continue
            ch = self._chan_of_slot(conn, chslot)
            if code == 404 and ch is not None:
                self._chan_close(c, ch, C.NOT_FOUND, "no exchange", 60, 40)
        for conn, status in seg_status:
            c = self.conns.get(conn)
            if c is None or c.state != "open":
                continue
            if status & SS_FRAME_ERROR:
                self._conn_close(c, C.FRAME_ERROR, "malformed frame")
            elif status & SS_UNEXPECTED:
                self._conn_close(c, C.UNEXPECTED_FRAME, "unexpected frame")
            elif status & SS_TOO_LARGE:
                self._conn_close(c, C.FRAME_ERROR, "command exceeds the server's limits")
            # SS_OVERFLOW is a per-step capacity limit: the rest stays in the carry
        for item in ctrl:
            conn, raw = item[0], item[1]
            # a step-decoded Basic.Get handed to the host did not pause its connection: its
            # answer must not resume one another command paused meanwhile
            dget = len(item) > 2 and item[2]
            c = self.conns.get(conn)
            if c is None:
                continue
            deferred = False
            if c.state == "open":
                self._dget_ctx = dget
                try:
                    deferred = self._control(c, raw) == "deferred"
                except _Hard as e:
                    self._conn_close(c, e.code, e.text, e.cls, e.mid)
                finally:
                    self._dget_ctx = False
            if c.state == "open" and not deferred and not dget:
                self._unpause(conn)
        return had_input or had_egress or bool(ctrl) or cnt.get("n_deliv", 0) > 0

    def _read_backpressure(self, segs):
        """Stop reading a connection while the device still holds a large backlog of its
        bytes (carry); resume once it drains."""
        carry = self.plane.carry
        # a connection's carry may legitimately grow to carry_cap (a large command being
        # assembled); stop reading only when the next read could overflow it
        lim = max(self.plane.info["carry_cap"] - self.per_conn_read, self.per_conn_read)
        for cid in segs["conn"]:
            cid = int(cid)
            big = carry[cid] > lim
            if big != (cid in self._rpaused):
                self.gw.set_read_paused(cid, big)
                (self._rpaused.add if big else self._rpaused.discard)(cid)
        for cid in list(self._rpaused):
            if carry[cid] <= lim:
                self.gw.set_read_paused(cid, False)
                self._rpaused.discard(cid)

    def _persist_step(self):
        """Store rows of this step, committed (fsync) before the step's egress — which
        carries its publisher confirms — leaves the broker."""
        if self.persistence is not None:
            self.persistence.after_step()
            self.persistence.commit()

    def _chan_of_slot(self, conn, chslot):
        cc = self.plane.conns.get(conn)
        if cc is None:
            return None
        for ch, chan in cc.channels.items():
            if conn * self.plane.chpc + chan.local == chslot:
                return ch
        return None

    def _unpause(self, conn):
        self.plane.unpause(conn)
        if self.fe is not None:
            self.fe.kick(conn)

    # ------------------------------------------------------------------ control methods
    def _control(self, c, raw):
        t, ch, size = struct.unpack_from(">BHI", raw, 0)
        if t != C.FRAME_METHOD:
            raise _Hard(C.UNEXPECTED_FRAME, "content frame without a method")
        m = decode_method(raw[7:7 + size])
        if self.ctl_trace is not None:   # (diagnostics: CHANAMQ_CTL_TRACE=1)
            self.ctl_trace.append((round(time.monotonic(), 4), c.id, ch, m.name, self.lock.deferring, self.lock.paused_at,
                                   getattr(m, "queue", None)))
        if ch in c.closing_channels:
            if m.name == "channel.close_ok":
                c.closing_channels.discard(ch)
            elif m.name == "channel.close":
                self._send(c, ch, Method("channel.close_ok"))
            return
        if ch == 0:
            return self._connection_method(c, m)
        p = self.plane
        chans = p.conns[c.id].channels
        if m.name == "channel.open":
            if ch in chans:
                raise _Hard(C.CHANNEL_ERROR, f"channel {ch} already open", 20, 10)
            if ch > self.channel_max:
                raise _Hard(C.CHANNEL_ERROR, f"channel {ch} above channel-max", 20, 10)
            try:
                p.open_channel(c.id, ch)
            except ControlError as e:
                raise _Hard(e.code, e.text, 20, 10)
            return self._send(c, ch, Method("channel.open_ok"))
        if ch not in chans:
            raise _Hard(C.CHANNEL_ERROR, f"channel {ch} is not open", m.class_id, m.method_id)
        if m.name == "basic.publish":   # the device hands over only publishes larger than its carry
            return self._big_begin(c, ch, m, raw, size)
        try:
            if self.node is not None and m.name in _REPLICATED_METHODS:
                return self._replicated(c, ch, m)
            r = self._channel_method(c, ch, m)
            if self.persistence is not None and m.name in _STORED_METHODS:
                # topology rows are durable before the *_ok reply leaves (c.out is
                # flushed after this command)
                self.persistence.control_commit()
            return r
        except ControlError as e:
            if e.code >= 500 or e.code in (C.CONNECTION_FORCED, C.INVALID_PATH):
                raise _Hard(e.code, e.text, e.class_id or m.class_id, e.method_id or m.method_id)
            self._chan_close(c, ch, e.code, e.text, m.class_id, m.method_id)

    # ------------------------------------------------------------------ large messages
    # A publish whose frames cannot fit the connection's device carry (64 MB bodies, say)
    # reaches the host as a control command (its method + header frames).  The host reads
    # the body frames -- the device's carry first, then the socket in host mode --, then
    # enqueues the message through the device's import path (GpuDataPlane.publish_host:
    # routed by its exchange, counted for the channel's confirms) and hands the connection
    # back to the data plane with whatever followed the body.
    def _big_begin(self, c, ch, m, raw, msize):
        p = self.plane
        hoff = 8 + msize
        _, _, hsize = struct.unpack_from(">BHI", raw, hoff)
        hp = bytes(raw[hoff + 7:hoff + 7 + hsize])
        _, body_size, props = decode_content_header(hp)
        vh = p.conns[c.id].vhost
        x = p.exchanges.get((vh, m.exchange))
        err = None
        if x is None:
            err = (C.NOT_FOUND, f"no exchange '{m.exchange}' in vhost '{vh}'")
        elif getattr(p.channel(c.id, ch), "tx", False):
            err = (C.NOT_IMPLEMENTED, "a message larger than the connection buffer inside a transaction")
        elif self.node is not None and self.fe is None:
            err = (C.NOT_IMPLEMENTED, "messages larger than the connection carry need the pipelined front end "
                                      "on a sharded node")
        elif body_size > p.max_host_message():
            err = (C.CONTENT_TOO_LARGE, f"message body of {body_size} bytes exceeds the broker's "
                                        f"{p.max_host_message()}-byte limit")
        c.big = dict(ch=ch, m=m, x=x, props=props, props_raw=hp[12:], size=body_size, body=bytearray(), got=0,
                     other=bytearray(), buf=bytearray(), err=err)
        c.state = "bigpub"
        carry = p.take_carry(c.id)
        if self.fe is not None:
            self.fe.set_host_mode(c.id)
        elif self.gw is not None:
            self.gw.set_data_mode(c.id, False)
        rest = self._big_feed(c, carry)
        if c.state == "open" and rest:   # (the body was already complete: cannot happen for a
            self._big_replay(c, rest)     # message larger than the carry, kept for safety)
        return "deferred"

    def _big_replay(self, c, rest):
        if self.fe is not None:
            self.fe.set_data_mode(c.id, rest)
        elif self.gw is not None:
            self.gw.set_data_mode(c.id, True)

    def _big_feed(self, c, data):
        """Host-mode bytes of a connection assembling a large publish; returns the bytes
        after it (frames of other channels read meanwhile first) once it is complete."""
        b = c.big
        b["buf"] += data
        buf, pos, done = b["buf"], 0, False
        while len(buf) - pos >= 8:
            t, fch, size = struct.unpack_from(">BHI", buf, pos)
            end = pos + 8 + size
            if len(buf) < end:
                break
            if buf[end - 1] != 0xCE:
                self._conn_close(c, C.FRAME_ERROR, "malformed frame")
                return b""
            if t == C.FRAME_BODY and fch == b["ch"]:
                if b["err"] is None:   # a rejected message is read and dropped
                    b["body"] += buf[pos + 7:end - 1]
                b["got"] += size
                if b["got"] > b["size"]:
                    self._conn_close(c, C.FRAME_ERROR, "body frames exceed the announced size")
                    return b""
            elif t == C.FRAME_HEARTBEAT:
                pass
            elif fch == b["ch"]:
                self._conn_close(c, C.UNEXPECTED_FRAME, "frame inside a message's content", 60, 40)
                return b""
            else:   # another channel's frame: replayed to the data plane after the message
                b["other"] += buf[pos:end]
            pos = end
            if b["got"] == b["size"]:
                done = True
                break
        if not done:
            del buf[:pos]
            return b""
        rest = bytes(b["other"]) + bytes(buf[pos:])
        return self._big_finish(c, rest)

    def _big_finish(self, c, rest=b""):
        """The body is complete: enqueue it.  Returns the bytes to hand back to the data
        plane now (a sharded node holds them until the message is in its queues)."""
        b, c.big = c.big, None
        c.state = "open"
        m, ch, props = b["m"], b["ch"], b["props"]
        if self.node is not None and b["err"] is None:
            return self._big_sharded(c, b, rest)
        with self.lock:
            if b["err"] is not None:
                code, text = b["err"]
                self._chan_close(c, ch, code, text, 60, 40)
            else:
                now = int(time.time() * 1000)
                flags = MF_PERSIST if props.get("delivery_mode") == 2 else 0
                ts = props.get("timestamp")
                ts_ms = int(ts) * 1000 if ts is not None else 0
                if ts is not None:
                    flags |= MF_HAS_TS
                exp = props.get("expiration")
                exp = exp.decode() if isinstance(exp, (bytes, bytearray)) else exp
                expire_ms = now + int(exp) if isinstance(exp, str) and exp.isdigit() else 0
                n = self.plane.publish_host(c.id, ch, b["x"].slot, m.exchange.encode(), m.routing_key.encode(),
                                           b["props_raw"], bytes(b["body"]), flags, expire_ms, ts_ms, now)
                self.stats["big_publishes"] = self.stats.get("big_publishes", 0) + 1
                if n == 0 and m.mandatory:
                    c.out += render_command(ch, Method("basic.return", reply_code=C.NO_ROUTE,
                                                       reply_text=C.REPLY_TEXT.get(C.NO_ROUTE, "NO_ROUTE"),
                                                       exchange=m.exchange, routing_key=m.routing_key),
                                            props, bytes(b["body"]), c.frame_max)
            self._unpause(c.id)
        self._flush(c)
        return rest

    @staticmethod
    def _big_meta(props):
        now = int(time.time() * 1000)
        flags = MF_PERSIST if props.get("delivery_mode") == 2 else 0
        ts = props.get("timestamp")
        ts_ms = int(ts) * 1000 if ts is not None else 0
        if ts is not None:
            flags |= MF_HAS_TS
        exp = props.get("expiration")
        exp = exp.decode() if isinstance(exp, (bytes, bytearray)) else exp
        expire_ms = now + int(exp) if isinstance(exp, str) and exp.isdigit() else 0
        return now, flags, expire_ms, ts_ms

    def _big_sharded(self, c, b, rest):
        """Sharded node: the queues the publish routes to may live on any rank.  Routed on
        the host over the replicated bindings, the message goes out as a control-log op
        whose body travels only to the owning ranks (ControlLog blob); at the sync every
        owner enqueues it into its queues and this rank counts it for the channel's
        confirms.  The connection stays off the data plane until then, so nothing it
        publishes later is confirmed or delivered ahead of it (FrameParser.scala:67: no
        size limit on any node)."""
        p, m, ch = self.plane, b["m"], b["ch"]
        x = b["x"]
        targets = {}
        for slot in p.route_host(x, m.routing_key.encode()):
            q = p.queue_by_slot.get(slot)
            if q is not None:
                targets.setdefault(int(q.owner), []).append(int(slot))
        now, flags, expire_ms, ts_ms = self._big_meta(b["props"])
        payload = m.exchange.encode() + m.routing_key.encode() + bytes(b["props_raw"]) + bytes(b["body"])
        meta = dict(origin=p.rank, conn=c.id, ch=ch, exch=x.slot, ex_len=len(m.exchange.encode()),
                    rk_len=len(m.routing_key.encode()), props_len=len(b["props_raw"]), body_len=len(b["body"]),
                    flags=flags, expire_ms=expire_ms, ts_ms=ts_ms, now=now,
                    targets={str(r): v for r, v in targets.items()})
        owners = sorted(set(targets) | {p.rank})
        with self.lock:
            seq = self.node.submit("big_publish", meta, blob=payload, blob_to=owners)
        self.stats["big_publishes"] = self.stats.get("big_publishes", 0) + 1
        c.state = "bigwait"
        c.big_rest = bytearray(rest)
        props, body = b["props"], bytes(b["body"])

        def reply(res, c=c):
            # the message is in its queues on every owner (this sync applied the op)
            if not targets and m.mandatory:
                c.out += render_command(ch, Method("basic.return", reply_code=C.NO_ROUTE,
                                                   reply_text=C.REPLY_TEXT.get(C.NO_ROUTE, "NO_ROUTE"),
                                                   exchange=m.exchange, routing_key=m.routing_key),
                                        props, body, c.frame_max)
            return None
        self._deferred[seq] = (c.id, ch, reply, m)
        return b""

    def _big_resume(self, c):
        """A sharded large publish was applied (or failed): the connection goes back to the
        data plane with the bytes that followed the message (_answer unpauses it)."""
        more = bytes(c.big_rest or b"")
        c.big_rest = None
        c.state = "open"
        self.fe.set_data_mode(c.id, more)

    def _apply_big(self, meta, blob=None):
        """Replicated ``big_publish`` (every rank, at the sync): the owners enqueue the
        message into their target queues; the origin's record also counts it for the
        publisher channel's confirms (and Nacks it if its store fails)."""
        p = self.plane
        mine = [int(s) for s in meta["targets"].get(str(p.rank), [])]
        origin = int(meta["origin"]) == p.rank
        if not (mine or origin) or blob is None:
            return 0
        el, rl, pl = meta["ex_len"], meta["rk_len"], meta["props_len"]
        ex, rk, props, body = blob[:el], blob[el:el + rl], blob[el + rl:el + rl + pl], blob[el + rl + pl:]
        n = 0
        if origin:   # routed by its exchange on this device: local queues + confirm counting
            n += p.publish_host(int(meta["conn"]), int(meta["ch"]), int(meta["exch"]), ex, rk, props,
                                body if mine else b"", int(meta["flags"]), int(meta["expire_ms"]),
                                int(meta["ts_ms"]), int(meta["now"]))
        else:
            n += p.publish_to_queues(mine, ex, rk, props, body, int(meta["flags"]), int(meta["expire_ms"]),
                                     int(meta["ts_ms"]), int(meta["now"]))
        return n

    def _connection_method(self, c, m):
        if m.name == "connection.close":
            self._send(c, 0, Method("connection.close_ok"))
            self._flush(c, direct=True)   # the connection's last bytes (fe.close follows)
            self._drop(c)
        elif m.name == "connection.close_ok":
            self._drop(c)
        else:
            raise _Hard(C.COMMAND_INVALID, f"unexpected {m.name}", m.class_id, m.method_id)

    def _channel_method(self, c, ch, m):
        p = self.plane
        vh = p.conns[c.id].vhost
        n = m.name
        if n == "channel.close":
            self._txbuf.pop((c.id, ch), None)
            p.close_channel(c.id, ch)
            if self._links:
                self._close_links(c.id, ch)
            self._send(c, ch, Method("channel.close_ok"))
        elif n == "channel.close_ok":
            pass
        elif n == "channel.flow":
            p.flow(c.id, ch, m.active)
            self._send(c, ch, Method("channel.flow_ok", active=m.active))
        elif n == "channel.flow_ok":
            pass
        elif n == "access.request":
            self._send(c, ch, Method("access.request_ok", ticket=1))
        elif n == "exchange.declare":
            if m.exchange.startswith("amq.") and not m.passive and (vh, m.exchange) not in p.exchanges:
                raise ControlError(C.ACCESS_REFUSED, f"exchange name '{m.exchange}' is reserved", 40, 10)
            x = p.exchanges.get((vh, m.exchange))
            if x is not None and not m.passive and x.type != m.type:
                raise ControlError(C.PRECONDITION_FAILED, f"exchange '{m.exchange}' declared as {x.type}", 40, 10)
            p.declare_exchange(vh, m.exchange, m.type or "direct", durable=m.durable, auto_delete=m.auto_delete,
                               internal=m.internal, arguments=m.arguments, passive=m.passive)
            if self.persistence is not None and not m.passive:
                self.persistence.exchange(p.exchanges[(vh, m.exchange)])
            if not m.nowait:
                self._send(c, ch, Method("exchange.declare_ok"))
        elif n == "exchange.delete":
            p.delete_exchange(vh, m.exchange, if_unused=m.if_unused)
            if self.persistence is not None:
                self.persistence.exchange_deleted(vh, m.exchange)
            if not m.nowait:
                self._send(c, ch, Method("exchange.delete_ok"))
        elif n == "queue.declare":
            name = m.queue or ("tmp." + uuid.uuid4().hex)
            args = m.arguments or {}
            ttl = int(args.get("x-message-ttl", 0) or 0)
            q = p.queues.get((vh, name))
            if q is not None and q.exclusive_owner not in (-1, c.id):
                raise ControlError(C.RESOURCE_LOCKED, f"queue '{name}' is exclusive to another connection", 50, 10)
            slot = p.declare_queue(vh, name, durable=m.durable, exclusive_owner=c.id if m.exclusive else -1,
                                   auto_delete=m.auto_delete, ttl_ms=ttl, passive=m.passive)
            c.last_queue[ch] = name
            if self.persistence is not None and q is None and not m.passive:
                self.persistence.queue(p.queue_by_slot[slot])
            if not m.nowait:
                qq = p.queue_by_slot[slot]
                cnt = 0 if q is None else p.message_count(slot)   # (a new queue: no device read)
                self._send(c, ch, Method("queue.declare_ok", queue=name, message_count=cnt,
                                         consumer_count=len(qq.consumers)))
        elif n == "queue.bind":
            qn = m.queue or c.last_queue.get(ch, "")
            p.bind(vh, qn, m.exchange, m.routing_key)
            if self.persistence is not None:
                self.persistence.bind(vh, qn, m.exchange, m.routing_key)
            if not m.nowait:
                self._send(c, ch, Method("queue.bind_ok"))
        elif n == "queue.unbind":
            qn = m.queue or c.last_queue.get(ch, "")
            p.unbind(vh, qn, m.exchange, m.routing_key)
            if self.persistence is not None:
                self.persistence.unbind(vh, qn, m.exchange, m.routing_key)
            self._send(c, ch, Method("queue.unbind_ok"))
        elif n == "queue.purge":
            q = self._queue(vh, m.queue or c.last_queue.get(ch, ""), 50, 30)
            cnt = p.purge(q.slot)
            if not m.nowait:
                self._send(c, ch, Method("queue.purge_ok", message_count=cnt))
        elif n == "queue.delete":
            q = self._queue(vh, m.queue or c.last_queue.get(ch, ""), 50, 40)
            if m.if_unused and q.consumers:
                raise ControlError(C.PRECONDITION_FAILED, f"queue '{q.name}' in use", 50, 40)
            cnt = p.message_count(q.slot)
            if m.if_empty and cnt:
                raise ControlError(C.PRECONDITION_FAILED, f"queue '{q.name}' not empty", 50, 40)
            p.purge(q.slot)
            # steps release the purged messages (front end paused); a deep durable queue
            # takes several: each step's TTL skip is bounded by its store-record buffer
            left = cnt
            while True:
                if self.fe is not None:
                    self._host_step({})
                else:
                    p.step({}, now_ms=int(time.time() * 1000))
                    self._persist_step()
                now_left = p.message_count(q.slot)
                if not now_left or now_left >= left:   # drained, or no progress (requeues)
                    break
                left = now_left
            p.delete_queue(vh, q.name)
            if self.persistence is not None:
                self.persistence.queue_deleted(vh, q.name, slot=q.slot)
            if not m.nowait:
                self._send(c, ch, Method("queue.delete_ok", message_count=cnt))
        elif n == "basic.qos":
            p.qos(c.id, ch, m.prefetch_count, m.prefetch_size, m.global_)
            self._send(c, ch, Method("basic.qos_ok"))
        elif n == "basic.consume":
            qn = m.queue or c.last_queue.get(ch, "")
            q = self._queue(vh, qn, 60, 20)
            tag = m.consumer_tag or ("amq.ctag-" + uuid.uuid4().hex)
            if self.node is not None and q.owner != p.rank:
                if (c.id, ch, tag) in self._links or tag in p.channel(c.id, ch).consumers:
                    raise ControlError(C.NOT_ALLOWED, f"consumer tag '{tag}' in use", 60, 20)
                return self._remote_consume(c, ch, vh, q, tag, m)
            p.consume(c.id, ch, vh, qn, tag, no_ack=m.no_ack)
            if not m.nowait:
                self._send(c, ch, Method("basic.consume_ok", consumer_tag=tag))
        elif n == "basic.cancel":
            p.cancel(c.id, ch, m.consumer_tag)
            if self._links:
                self._close_links(c.id, ch, m.consumer_tag)
            if not m.nowait:
                self._send(c, ch, Method("basic.cancel_ok", consumer_tag=m.consumer_tag))
        elif n in ("basic.recover", "basic.recover_async"):
            p.recover(c.id, ch)   # requeue=false is treated as requeue (RabbitMQ behaviour)
            if n == "basic.recover":
                self._send(c, ch, Method("basic.recover_ok"))
        elif n == "confirm.select":
            if p.channel(c.id, ch).tx:
                raise ControlError(C.PRECONDITION_FAILED, "cannot switch from tx to confirm mode", 85, 10)
            p.confirm_select(c.id, ch)
            if self.fe is not None and self.confirm_read:
                self.fe.set_read_cap(c.id, min(self.confirm_read, self.per_conn_read))
            if not m.nowait:
                self._send(c, ch, Method("confirm.select_ok"))
        elif n == "basic.get":
            q = self._queue(vh, m.queue or c.last_queue.get(ch, ""), 60, 70)
            if q.exclusive_owner not in (-1, c.id):
                raise ControlError(C.RESOURCE_LOCKED, f"queue '{q.name}' is exclusive to another connection", 60, 70)
            if q.owner != p.rank:
                return self._remote_get(c, ch, vh, q, m)
            if self.fe is not None and hasattr(p, "eng"):
                # served inside the next step (k_dequeue, ahead of the queue's consumers): no
                # pipeline drain; the connection stays paused until FE_GET answers it
                gid = self._next_get = getattr(self, "_next_get", 0) + 1
                self._dev_gets[gid] = (c.id, ch, q.slot, bool(m.no_ack), vh, q.name, not self._dget_ctx)
                self.fe.queue_get(c.id, p.chslot(c.id, ch), q.slot, int(bool(m.no_ack)), gid)
                self.stats["device_gets"] = self.stats.get("device_gets", 0) + 1
                return "deferred"
            frames, _ = p.basic_get(c.id, ch, q.slot, m.no_ack, int(time.time() * 1000))
            if frames is None:
                self._send(c, ch, Method("basic.get_empty"))
            else:
                c.out += frames
        elif n == "tx.select":
            if p.channel(c.id, ch).confirm:
                raise ControlError(C.PRECONDITION_FAILED, "cannot switch from confirm to tx mode", 90, 10)
            if not p.channel(c.id, ch).tx:
                p.tx_select(c.id, ch)
                self._txbuf[(c.id, ch)] = []
            self._send(c, ch, Method("tx.select_ok"))
        elif n in ("tx.commit", "tx.rollback"):
            if not p.channel(c.id, ch).tx:
                raise ControlError(C.PRECONDITION_FAILED, "channel is not transactional", 90, m.method_id)
            if n == "tx.rollback":
                self._txbuf[(c.id, ch)] = []
                self._send(c, ch, Method("tx.rollback_ok"))
            else:
                return self._tx_commit(c, ch)
        elif n in ("exchange.bind", "exchange.unbind"):
            raise ControlError(C.NOT_IMPLEMENTED, f"{n} is not served by the GPU data path", m.class_id,
                               m.method_id)
        elif n == "basic.publish":   # publish on a channel the device did not know (closing race)
            raise ControlError(C.CHANNEL_ERROR, "publish on a closed channel", 60, 40)
        else:
            raise _Hard(C.COMMAND_INVALID, f"unexpected {n}", m.class_id, m.method_id)

    # ------------------------------------------------------------------ sharded control ops
    def _replicated(self, c, ch, m):
        """Submit a replicated op to the control log; the reply (and the unpause of the
        connection) happens in the step that applies it on every rank."""
        p, node = self.plane, self.node
        vh = p.conns[c.id].vhost
        n = m.name
        if n == "exchange.declare":
            x = p.exchanges.get((vh, m.exchange))
            if m.passive:
                if x is None:
                    raise ControlError(C.NOT_FOUND, f"no exchange '{m.exchange}' in vhost '{vh}'", 40, 10)
                return self._send(c, ch, Method("exchange.declare_ok"))
            if m.exchange.startswith("amq.") and x is None:
                raise ControlError(C.ACCESS_REFUSED, f"exchange name '{m.exchange}' is reserved", 40, 10)
            if x is not None and x.type != m.type:
                raise ControlError(C.PRECONDITION_FAILED, f"exchange '{m.exchange}' declared as {x.type}", 40, 10)
            seq = node.submit("declare_exchange", vh, m.exchange, m.type or "direct", durable=m.durable,
                              auto_delete=m.auto_delete, internal=m.internal, arguments=dict(m.arguments or {}))
            reply = None if m.nowait else (lambda r: Method("exchange.declare_ok"))
        elif n == "exchange.delete":
            seq = node.submit("delete_exchange", vh, m.exchange, if_unused=m.if_unused)
            reply = None if m.nowait else (lambda r: Method("exchange.delete_ok"))
        elif n == "queue.declare":
            name = m.queue or ("tmp." + uuid.uuid4().hex)
            q = p.queues.get((vh, name))
            if m.passive:
                if q is None:
                    raise ControlError(C.NOT_FOUND, f"no queue '{name}' in vhost '{vh}'", 50, 10)
                c.last_queue[ch] = name
                cnt = p.message_count(q.slot) if q.owner == p.rank else 0
                return self._send(c, ch, Method("queue.declare_ok", queue=name, message_count=cnt,
                                                consumer_count=len(q.consumers)))
            if q is None:   # client-local placement: the queue lives on the declaring rank
                node.submit("place_queue", vh, name, p.rank)
            args = m.arguments or {}
            seq = node.submit("declare_queue", vh, name, durable=m.durable, auto_delete=m.auto_delete,
                              ttl_ms=int(args.get("x-message-ttl", 0) or 0))
            c.last_queue[ch] = name

            def reply(r, name=name):
                qq = p.queues.get((vh, name))
                return Method("queue.declare_ok", queue=name, message_count=0,
                              consumer_count=len(qq.consumers) if qq else 0)
            reply = None if m.nowait else reply
        elif n in ("queue.bind", "queue.unbind"):
            qn = m.queue or c.last_queue.get(ch, "")
            seq = node.submit("bind" if n == "queue.bind" else "unbind", vh, qn, m.exchange, m.routing_key)
            ok = "queue.bind_ok" if n == "queue.bind" else "queue.unbind_ok"
            reply = None if (n == "queue.bind" and m.nowait) else (lambda r, ok=ok: Method(ok))
        else:   # queue.delete
            q = self._queue(vh, m.queue or c.last_queue.get(ch, ""), 50, 40)
            if m.if_unused and q.consumers:
                raise ControlError(C.PRECONDITION_FAILED, f"queue '{q.name}' in use", 50, 40)
            seq = node.submit("delete_queue", vh, q.name)
            reply = None if m.nowait else (lambda r: Method("queue.delete_ok", message_count=0))
        self._deferred[seq] = (c.id, ch, reply, m)
        return "deferred"

    def _answer(self, results):
        """Replies for this rank's control-log ops applied in this step."""
        from ..parallel.control_log import error_of
        pending, self._deferred = self._deferred, {}
        for seq, (conn, ch, reply, m) in pending.items():
            c = self.conns.get(conn)
            if c is None or c.state not in ("open", "bigwait"):
                if hasattr(reply, "abandon"):   # e.g. a link opened for a connection now gone
                    reply.abandon()
                continue
            res = results.get(seq)
            err = error_of(res)
            if c.state == "bigwait":
                self._big_resume(c)
            if err:
                code, text, cls, mid = err
                if code >= 500:
                    self._conn_close(c, code, text, cls or m.class_id, mid or m.method_id)
                    continue
                self._chan_close(c, ch, code, text, m.class_id, m.method_id)
            elif reply is not None:
                out = reply(res)
                if out is not None:
                    self._send(c, ch, out)
            if c.state == "open" and not (hasattr(reply, "keep_paused") and reply.keep_paused(res)):
                self._unpause(conn)

    def _get_answer(self, conn, a, gid):
        """FE_GET: the step that carried Basic.Get ``gid`` finished.  OK: its GetOk + header
        + body were rendered into the connection's egress of that step; EMPTY: GetEmpty
        from here; RETRY (the step was full): with the next step."""
        req = self._dev_gets.pop(gid, None)
        c = self.conns.get(conn)
        if req is None or c is None or c.state != "open":
            return
        st, cnt = a & 0xFFFFFFFF, a >> 32
        _, ch, slot, no_ack, vh, qname, resume = req
        q = self.plane.queues.get((vh, qname))
        if st == GS_RETRY and (q is None or q.slot != slot or q.owner != self.plane.rank):
            st = GS_GONE   # deleted (or moved) while the Get waited: never resubmitted
        if st == GS_RETRY:
            self._dev_gets[gid] = req
            self.fe.queue_get(conn, self.plane.chslot(conn, ch), slot, int(no_ack), gid)
            return
        if st == GS_GONE:   # the reference's Pull on a missing queue entity: 404
            self._chan_close(c, ch, C.NOT_FOUND, f"no queue '{qname}' in vhost '{vh}'", 60, 70)
        elif st == GS_EMPTY:
            self._send(c, ch, Method("basic.get_empty"))
        elif st != GS_OK:
            self._chan_close(c, ch, C.RESOURCE_ERROR, "basic.get: " + (
                "message exceeds the egress buffer" if st == GS_NO_SPACE else "channel delivery window full"), 60, 70)
        self._flush(c)
        if c.state == "open" and resume:
            self._unpause(conn)

    def _remote_get(self, c, ch, vh, q, m):
        """Basic.Get of a queue another rank owns: a pull on this rank's get link for the
        queue (opened on first use, closed when idle); the owner's answer comes back after
        the step and ``_serve_gets`` replies (parallel/links.py)."""
        p, links = self.plane, self.node.links
        key = (vh, q.name)
        lid = self._get_links.get(key)
        lk = links.links.get(lid) if lid is not None else None
        if lk is not None and lk.closing:
            lid = lk = None
        if lk is not None and not lk.pending and not any(w[3] == lid for w in self._get_wait.values()):
            sq = p.queues.get((vh, lk.shadow))
            if sq is not None and p.message_count(sq.slot):   # a requeued one is still here
                self._get_used[lid] = time.monotonic()
                self._serve_get(c, ch, m.no_ack, lid, None)
                return None
        if lid is None:
            self._link_seq += 1
            lid = (p.rank << 24) | self._link_seq
            self.node.submit("link_open", lid, vh, q.name, p.rank, 0, get=True)
            self._get_links[key] = lid
        self._pull_seq += 1
        pn = (p.rank << 40) | self._pull_seq
        seq = self.node.submit("link_pull", lid, pn)
        self._get_wait[pn] = (c.id, ch, bool(m.no_ack), lid)
        self._get_used[lid] = time.monotonic()

        def reply(res, pn=pn, lid=lid, key=key):
            if res is False:   # the link is gone (or never opened): nothing to get
                self._get_wait.pop(pn, None)
                if self._get_links.get(key) == lid and lid not in self.node.links.links:
                    self._get_links.pop(key, None)
                return Method("basic.get_empty")
            return None
        reply.keep_paused = lambda res: res is not False   # until the owner's answer
        reply.abandon = lambda pn=pn: self._get_wait.pop(pn, None)
        self._deferred[seq] = (c.id, ch, reply, m)
        return "deferred"

    def _serve_get(self, c, ch, no_ack, lid, cnt):
        """Answer a Get from the get link's shadow queue (the message the owner sent is
        there once ``links.before_step`` ran): GetOk with this channel's delivery tag and
        the owner's remaining count."""
        from ..parallel.links import set_get_ok_count
        p = self.plane
        lk = self.node.links.links.get(lid)
        sq = p.queues.get((lk.vhost, lk.shadow)) if lk is not None else None
        frames = None
        if sq is not None:
            try:
                frames, left = p.basic_get(c.id, ch, sq.slot, False)
            except (ControlError, KeyError):
                frames = None
        if frames is None:
            self._send(c, ch, Method("basic.get_empty"))
            return
        frames = set_get_ok_count(frames, left if cnt is None else cnt)
        if no_ack:   # consumed now: the shadow's consumed record acks it at the owner
            p.apply_ack(c.id, ch, struct.unpack_from(">Q", frames, 11)[0])
        else:
            self._get_holders.setdefault(lid, set()).add((c.id, ch))
        c.out += frames

    def _serve_gets(self):
        """Before a step: answers that came back for remote Gets; close get links idle
        for a second with nobody holding their messages (what a closed link held goes
        back to the owner's queue)."""
        links = self.node.links
        links.before_step()
        for pn, lid, cnt in links.take_gets():
            w = self._get_wait.pop(pn, None)
            if w is None:
                continue
            conn, ch, no_ack, _ = w
            c = self.conns.get(conn)
            if c is None or c.state != "open" or ch in c.closing_channels:
                continue
            if cnt is None:
                self._send(c, ch, Method("basic.get_empty"))
            else:
                self._serve_get(c, ch, no_ack, lid, cnt)
            self._unpause(conn)
        if not self._get_links:
            return
        now = time.monotonic()
        waiting = {w[3] for w in self._get_wait.values()}
        for key, lid in list(self._get_links.items()):
            if lid in waiting or now - self._get_used.get(lid, 0.0) < 1.0:
                continue
            pc = self.plane.conns
            hold = {(cn, ch) for cn, ch in self._get_holders.get(lid, ())
                    if cn in self.conns and self.conns[cn].state == "open"
                    and ch not in self.conns[cn].closing_channels and cn in pc and ch in pc[cn].channels}
            if hold:
                self._get_holders[lid] = hold
                continue
            self._get_links.pop(key)
            self._get_holders.pop(lid, None)
            self._get_used.pop(lid, None)
            if lid in links.links:
                self.node.submit("link_close", lid)

    def _alloc_link_slot(self):
        if not self._link_free:
            raise ControlError(C.RESOURCE_ERROR, "no connection slot left for a remote consumer", 60, 20)
        return self._link_free.pop()

    def _remote_consume(self, c, ch, vh, q, tag, m):
        """Basic.Consume of a queue another rank owns (X2/X3): a link through the control
        log; once applied on every rank the client's consumer attaches here to the link's
        shadow queue (parallel/links.py)."""
        p = self.plane
        self._link_seq += 1
        lid = (p.rank << 24) | self._link_seq
        pf = p.channel(c.id, ch).prefetch_count
        seq = self.node.submit("link_open", lid, vh, q.name, p.rank, 0 if m.no_ack else pf)

        def reply(res, lid=lid):
            shadow = self.node.links.shadow_of(lid)
            try:
                p.consume(c.id, ch, vh, shadow, tag, no_ack=m.no_ack)
            except ControlError as e:
                self.node.submit("link_close", lid)
                self._chan_close(c, ch, e.code, e.text, 60, 20)
                return None
            self._links[(c.id, ch, tag)] = lid
            return None if m.nowait else Method("basic.consume_ok", consumer_tag=tag)
        reply.abandon = lambda lid=lid: self.node.submit("link_close", lid)
        self._deferred[seq] = (c.id, ch, reply, m)
        return "deferred"

    def _close_links(self, conn, ch=None, tag=None):
        """Cancel / channel close / connection close of remote consumers."""
        for key in [k for k in self._links if k[0] == conn and (ch is None or k[1] == ch)
                    and (tag is None or k[2] == tag)]:
            self.node.submit("link_close", self._links.pop(key))

    def _queue(self, vh, name, cls, mid):
        q = self.plane.queues.get((vh, name))
        if q is None:
            raise ControlError(C.NOT_FOUND, f"no queue '{name}' in vhost '{vh}'", cls, mid)
        return q

    # ------------------------------------------------------------------ output
    def _send(self, c, ch, m):
        c.out += encode_method_frame(ch, m)

    def _chan_close(self, c, ch, code, text, cls, mid):
        self.plane.close_channel(c.id, ch)
        if self._links:
            self._close_links(c.id, ch)
        c.closing_channels.add(ch)
        self._send(c, ch, Method("channel.close", reply_code=code, reply_text=text[:255], class_id=cls,
                                 method_id=mid))

    def _conn_close(self, c, code, text, cls=0, mid=0):
        if c.state in ("closing", "closed"):
            return
        self._send(c, 0, Method("connection.close", reply_code=code, reply_text=text[:255], class_id=cls,
                                method_id=mid))
        if self._links:
            self._close_links(c.id)
        with self.lock:
            self.plane.close_connection(c.id)
            if self.fe is not None:   # its bytes go to the host again (waiting for CloseOk)
                self._flush(c)
                self.fe.set_host_mode(c.id)
        c.state = "closing"

    def _flush(self, c, direct=False):
        if not c.out or c.state == "closed":
            return
        if self.fe is not None:
            if self.ctl_trace is not None:
                self.ctl_trace.append((round(time.monotonic(), 4), c.id, "flush", len(c.out),
                                       self.lock.deferring and c.state == "open" and not direct))
            if self.lock.deferring and c.state == "open" and not direct:
                # behind the deliveries of the steps in flight and the step carrying this
                # command's table writes
                self.fe.send_after(c.id, bytes(c.out))
            else:
                self.fe.send(c.id, bytes(c.out))
            c.out.clear()
            c.last_tx = time.monotonic()
            return
        if self.gw is not None:
            self.gw.send(c.id, bytes(c.out))
            c.out.clear()
            c.last_tx = time.monotonic()
            return
        try:
            n = c.sock.send(c.out)
        except (BlockingIOError, InterruptedError):
            return
        except OSError:
            self._drop(c)
            return
        del c.out[:n]
        c.last_tx = time.monotonic()

    def _flush_all(self):
        for c in list(self.conns.values()):
            if c.out:
                self._flush(c)

    def _watermarks(self):
        # a failed store never accepts another persistent publish: publishers are blocked for
        # good (Connection.Blocked / Channel.Flow off) and the front end turns every confirm it
        # still held into Basic.Nack (frontend.cpp collect_scatter); /admin/stats reports it
        if "store_failed" in self.stats:
            if not self.blocked:
                self.blocked = True
                self.stats["flow_off"] = self.stats.get("flow_off", 0) + 1
                self._set_flow(False)
            return
        if self.spill_at:
            self._maybe_spill()
        if self.cold is not None and getattr(self, "_cold_thread", None) is None:
            self._maybe_cold()
        if not self.mem_high:
            return
        if self.fe is not None and self._fe_stats:
            used, msgs, logu = self._fe_stats["live_bytes"], self._fe_stats["live_msgs"], self._fe_stats["log_used"]
        else:
            lc = getattr(self.plane, "last_counters", None) or {}
            used, msgs = self.plane.memory_in_use(), lc.get("n_live_msgs", 0)
            logu = lc.get("log_head", 0) - lc.get("log_tail", 0)
        high = used >= self.mem_high or (self.msg_high and msgs >= self.msg_high) or \
            (self.log_high and logu >= self.log_high)
        low = used <= self.mem_low and (not self.msg_high or msgs <= self.msg_low) and \
            (not self.log_high or logu <= self.log_low)
        if not self.blocked and high:
            self.blocked = True
            self.stats["flow_off"] = self.stats.get("flow_off", 0) + 1
            self._set_flow(False)
        elif self.blocked and low:
            self.blocked = False
            self._set_flow(True)

    def _maybe_spill(self):
        if self.fe is not None and self._fe_stats:
            logu = self._fe_stats["log_used"]
        else:
            lc = getattr(self.plane, "last_counters", None) or {}
            logu = lc.get("log_head", 0) - lc.get("log_tail", 0)
        if self.fe is not None and hasattr(self.plane, "eng") and self.node is None:
            # pipelined single-GPU engine: above the watermark every step moves its share
            # (k_dequeue, at most 2 MiB a step so the egress D2H keeps most of the link) --
            # no pipeline drain; _sync_fe_stats counts the bytes
            on = logu >= self.spill_at
            if on != getattr(self, "_spill_on", False):
                self._spill_on = on
                self.plane.eng.stage_spill(1 << 15 if on else 0, self.spill_hot, 2 << 20)
                if on:
                    self.fe.wake()
            return
        now = time.monotonic()
        if logu < self.spill_at or now - self._last_spill < 0.01:
            return
        self._last_spill = now
        with self.lock:
            moved = self.plane.spill(0.5, self.spill_hot)
        if moved:
            self.stats["spilled_bytes"] = self.stats.get("spilled_bytes", 0) + moved
            self.stats["spills"] = self.stats.get("spills", 0) + 1

    def _maybe_cold(self):
        """Cold tier upkeep (at most every 10 ms): page the bodies near the held queues'
        heads back in, move cold spilled bodies out once the ring is 60% full, and unlink
        released store segments (every second)."""
        now = time.monotonic()
        if now - self._last_cold < 0.01:
            return
        self._last_cold = now
        p = self.plane
        sb = p.info["spill_bytes"]
        if self._cold_pending:
            with self.lock:
                got = p.cold_in(self.cold, self.cold_window)
            self.stats["cold_in_bytes"] = self.stats.get("cold_in_bytes", 0) + got
        if p.spill_used() > 0.6 * sb:
            with self.lock:
                moved = p.cold_out(self.cold, self.cold_hot, sb // 4)
            if moved:
                self._cold_pending = True
                self.stats["cold_out_bytes"] = self.stats.get("cold_out_bytes", 0) + moved
                self.stats["cold_outs"] = self.stats.get("cold_outs", 0) + 1
        if self._cold_pending and now - self._last_cold_gc > 1.0:
            self._last_cold_gc = now
            live = p.cold_live()
            self.cold.gc(live)
            self._cold_pending = bool((live > 0).any())

    def _cold_beside(self):
        """The cold tier runs beside the steps (its own thread, engine side operations)
        on a single-GPU engine driven by the native front end."""
        return (self.cold_beside and self.cold is not None and self.fe is not None and self.node is None
                and hasattr(getattr(self.plane, "eng", None), "side_cold_pick"))

    def _side(self, post):
        """Post one engine side operation, wake the stepper (an idle broker submits a step
        for it) and wait for its result; the steps never wait for the store."""
        post()
        self.fe.wake()
        while True:
            r = self.plane.eng.side_wait(0.05)
            if r is not None:
                self.stats["cold_side_ops"] = self.stats.get("cold_side_ops", 0) + 1
                return r
            if not self._running:
                raise _ColdStopped()

    def _cold_loop(self):
        """_maybe_cold beside the steps: every 10 ms page the bodies near held queues'
        heads back in and move cold spilled bodies out once the ring is 60% full (the
        device checks the fill), every second unlink released store segments -- no
        stepper pause."""
        p = self.plane
        sb = p.info["spill_bytes"]
        last_gc = 0.0
        while self._running:
            time.sleep(0.01)
            if not self._cold_pending and not self.stats.get("spilled_bytes", 0):
                continue   # nothing ever left HBM: no side operation (each costs a step launch)
            try:
                if self._cold_pending:
                    got = p.cold_in_side(self.cold, self._side, self.cold_window)
                    self.stats["cold_in_bytes"] = self.stats.get("cold_in_bytes", 0) + got
                moved = p.cold_out_side(self.cold, self._side, self.cold_hot, sb // 4)
                if moved:
                    self._cold_pending = True
                    self.stats["cold_out_bytes"] = self.stats.get("cold_out_bytes", 0) + moved
                    self.stats["cold_outs"] = self.stats.get("cold_outs", 0) + 1
                now = time.monotonic()
                if self._cold_pending and now - last_gc > 1.0:
                    last_gc = now
                    live = p.cold_live_side(self._side)
                    self.cold.gc(live)
                    self._cold_pending = bool((live > 0).any())
            except _ColdStopped:
                return
            except Exception as e:   # (kept running: a store error must not end the tier)
                self.stats["cold_errors"] = self.stats.get("cold_errors", 0) + 1
                logging.getLogger("chanamq.gpu").warning("cold tier: %s", e)
                try:   # an operation posted before the error still completes first
                    while self._running and self.plane.eng.side_pending():
                        self.plane.eng.side_wait(0.05)
                except Exception:
                    pass
                time.sleep(0.1)

    def _set_flow(self, active):
        for c in list(self.conns.values()):
            if c.state != "open":
                continue
            if c.cap_blocked:
                if active:
                    self._send(c, 0, Method("connection.unblocked"))
                else:
                    self._send(c, 0, Method("connection.blocked", reason="persistent store failed"
                                            if "store_failed" in self.stats else "low on memory"))
            else:
                pc = self.plane.conns.get(c.id)
                for ch in (list(pc.channels) if pc else []):
                    if ch not in c.closing_channels:
                        self._send(c, ch, Method("channel.flow", active=active))

    def _heartbeats(self, now):
        for c in list(self.conns.values()):
            if c.state != "open" or not c.heartbeat:
                continue
            if now - c.last_tx >= c.heartbeat / 2 and not c.out:
                c.out += HEARTBEAT
            if now - c.last_rx > 2 * c.heartbeat:   # missed two heartbeats: peer is gone
                self._drop(c)

    def _drop(self, c):
        if c.state == "closed":
            return
        prev = c.state
        c.state = "closed"
        if self._links:
            self._close_links(c.id)
        if self.fe is not None:
            self.fe.cancel_gets(c.id)
            for gid in [g for g, r in self._dev_gets.items() if r[0] == c.id]:
                del self._dev_gets[gid]
            if prev != "gone":
                self._flush(c)
            if prev == "open" or c.id in self.plane.conns:
                light = self.lock.deferring or (self._light_capable() and self._close_light(c))
                with (self.light if light and self._close_light(c) else self.lock):
                    self.plane.close_connection(c.id)
            self.conns.pop(c.id, None)
            self.fe.close(c.id)
            return
        if self.gw is not None:
            if prev != "gone":
                self._flush(c)
                self.gw.flush()
                self.gw.close(c.id)
        else:
            try:
                self._sel.unregister(c.sock)
            except (KeyError, ValueError):
                pass
            try:
                c.sock.close()
            except OSError:
                pass
        if prev in ("open",) or c.id in self.plane.conns:
            with self.lock:
                self.plane.close_connection(c.id)
        self.conns.pop(c.id, None)
        if self.gw is None:
            self._free.append(c.id)


__all__ = ["GpuBroker", "encode_table"]
