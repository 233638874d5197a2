"""One rank of a sharded broker: data plane + communicator + replicated control log +
failure detector, stepped in lockstep with its peers.

  step(inputs):  control-log sync (all-gather, apply everywhere)
                 -> data-plane step (phase A, all-to-all of cross-rank publishes, phase B)
  on a failed collective:  wait for the failure detector, agree on the dead set, rebuild
                 the communicator over the survivors, re-home the dead ranks' queues
                 (rendezvous hashing moves only those), retry the step.

This is the reference's cluster behaviour (Akka cluster sharding re-homes entities of a
downed node) for the per-step collective design.  Messages held only by the
dead GPU are lost unless persistent on durable queues (reloaded from the store by the
new owner).
"""

import logging

from .comm import Comm
from .control_log import ControlLog
from .exchange import Exchanger
from .links import RemoteLinks
from .membership import Membership

log = logging.getLogger("chanamq.node")


class ShardedNode:
    def __init__(self, plane, comm: Comm = None, membership: Membership = None, hb_timeout_s=2.0,
                 persistence=None, peer_store=None):
        """persistence: this rank's GpuPersistence; peer_store(rank) -> an opened Store of
        that rank's (shared-filesystem) store directory, used to adopt the durable queues
        of a dead rank (``handle_failure``)."""
        self.plane = plane
        self.persistence, self.peer_store = persistence, peer_store
        self.comm = comm or Comm()
        self.exchanger = Exchanger(self.comm)
        plane.exchanger = None   # the node drives the exchange (and retries it on failover)
        self.log = ControlLog(plane, self.comm)
        self.members = membership or Membership(self.comm.store, self.comm.rank, self.comm.world,
                                                timeout_s=hb_timeout_s)
        self.failovers = []
        self.fe = None              # native front end (pipelined sharded server)
        self.rebuild_xchg = None    # (live ranks, epoch) -> rebuild the engine's exchange
        # remote consumers (X2/X3): link ops ride the control log, link traffic one
        # all-to-all after each data step while links exist
        self.links = RemoteLinks(plane)
        self.log.handlers["link_open"] = self.links.open
        self.log.handlers["link_close"] = self.links.close
        self.log.handlers["link_pull"] = self.links.pull

    @property
    def rank(self):
        return self.comm.rank

    def submit(self, op, *args, **kw):
        seq = self.log.submit(op, *args, **kw)
        if self.fe is not None:   # every rank syncs at the next step (frontend.cpp XF_SYNC)
            self.fe.request_sync()
        return seq

    # ------------------------------------------------------------------ pipelined server
    def use_device_links(self, alloc_conn, free_conn):
        """Remote consumers through the data plane (X2/X3 records in the exchange) instead
        of the host relay: the pipelined server has no per-step host collective."""
        from .links import DeviceLinks
        self.links = DeviceLinks(self.plane, alloc_conn, free_conn, self.submit)
        self.log.handlers["link_open"] = self.links.open
        self.log.handlers["link_close"] = self.links.close
        self.log.handlers["link_pull"] = self.links.pull
        self.log.handlers["link_got"] = self.links.got_answer

    def attach_frontend(self, fe, stuck_s=5.0):
        """The native front end steps this rank (frontend.cpp stepper_sharded): control
        ops sync at its FE_SYNC points, failovers run at FE_XFAIL, and this rank's
        heartbeat only beats while the stepper makes progress (a wedged GPU or a failed
        engine stops it, so the peers fail this rank over instead of hanging on it)."""
        self.fe = fe
        self.members.health = lambda: fe.healthy(stuck_s)

    def sync_point(self):
        """All ranks parked at the same step: the control log all-gather (on the host
        control group) applied everywhere -> {seq: result} of this rank's ops."""
        return self._retry(self.log.sync, 3)

    def failover_point(self):
        """An exchange peer stopped answering: agree on the dead ranks, rebuild the
        communicators (control group and the engine's exchange) over the survivors,
        re-home the dead ranks' queues and reload their durable messages."""
        return self.handle_failure()

    def step(self, inputs=None, now_ms=0, retries=3):
        """One lockstep step -> (plane step result, {seq: result} of this rank's ops)."""
        self.links.before_step()
        results = self._retry(self.log.sync, retries)
        res = self._data_step(inputs or {}, now_ms, retries)
        self.relay(res["egress"] if isinstance(res, dict) else res.egress, retries)
        return res, results

    def relay(self, egress, retries=3):
        """After a data step: owner-side deliveries of the remote consumers' pseudo
        connections (taken out of ``egress``) and connection-side acks, one all-to-all."""
        if not self.links.active:
            return
        out = self.links.outgoing(egress)
        got = self._retry(lambda: self.comm.alltoall_bytes(out), retries)
        self.links.incoming(got)
        self.links.after_step()

    def step_raw(self, segs, ptr, nbytes, now_ms, retries=3):
        """GPU plane, pre-staged ingress (server gateway): runs phase A, the exchange and
        phase B; returns (ticket for plane.finish, {seq: result}).  The caller runs
        ``relay`` with the pseudo connections' egress once the step finished."""
        self.links.before_step()
        results = self._retry(self.log.sync, retries)
        p = self.plane
        ticket = p.submit_raw(segs, ptr, nbytes, now_ms)
        recv = self._retry(lambda: self.exchanger.exchange(p.pending_send_counts(), p.xfer_send_desc(),
                                                           p.xfer_send_pay(), p.xfer_recv_desc(),
                                                           p.xfer_recv_pay()), retries)
        if p.lag:
            p.set_import(recv)
        else:
            p.submit_b(recv)
        return ticket, results

    def _retry(self, fn, retries):
        for attempt in range(retries + 1):
            try:
                return fn()
            except RuntimeError as e:   # a peer vanished mid-collective
                if attempt == retries:
                    raise
                log.warning("rank %d: collective failed (%s); checking membership", self.rank, e)
                self.handle_failure()

    def _data_step(self, inputs, now_ms, retries):
        p = self.plane
        gpu = hasattr(p, "eng")
        # a connection the control-log sync just closed (or that closed while its bytes
        # were gathered) takes no part in the step
        inputs = {c: v for c, v in inputs.items() if c in p.conns}
        if gpu:
            segs, ptr, n = p.stage(inputs)
            ticket = p.submit_raw(segs, ptr, n, now_ms)     # phase A (no exchanger on the plane)
        else:
            p.step_a(inputs, now_ms)
        recv = self._retry(lambda: self.exchanger.exchange(p.pending_send_counts(), p.xfer_send_desc(),
                                                           p.xfer_send_pay(), p.xfer_recv_desc(),
                                                           p.xfer_recv_pay()), retries)
        if gpu:
            if p.lag:
                p.set_import(recv)
            else:
                p.submit_b(recv)
            return p.finish(ticket)
        return p.step_b(recv)

    def handle_failure(self, suspects=None):
        suspects = suspects if suspects is not None else self.members.wait_suspects()
        if not suspects:
            raise RuntimeError("collective failed but no peer is suspected")
        dead = self.members.agree_dead(suspects, epoch=self.comm.epoch + 1)
        self.comm.rebuild(self.members.live)
        if self.rebuild_xchg is not None:
            self.rebuild_xchg(sorted(self.members.live), self.comm.epoch)
        for r in dead:
            self.plane.shard_map.fail(r)
        self.links.on_failure(dead)
        prev = {q.slot: q.owner for q in self.plane.queue_by_slot.values()}
        moved = self.plane.rehome(dead)
        self.links.after_rehome()
        adopted = self._adopt(dead, prev)
        self.failovers.append((sorted(dead), moved, adopted))
        log.warning("rank %d: ranks %s left; re-homed %d queues, reloaded %d durable messages",
                    self.rank, sorted(dead), len(moved), adopted)
        return dead, moved

    def _adopt(self, dead, prev):
        """Durable queues that moved here from a dead rank: reload their stored messages
        from that rank's store (the reference's re-homed QueueEntity reloads from
        Cassandra)."""
        if self.persistence is None or self.peer_store is None:
            return 0
        n = 0
        for r in sorted(dead):
            mine = [q for q in self.plane.queue_by_slot.values()
                    if prev.get(q.slot) == r and q.owner == self.rank and q.durable]
            if not mine:
                continue
            src = self.peer_store(r)
            try:
                n += self.persistence.adopt(src, mine)
            finally:
                src.close()
        return n

    def close(self):
        self.members.stop()
