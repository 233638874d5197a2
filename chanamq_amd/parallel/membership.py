"""Rank membership and failure detection (the role of Akka Cluster's gossip + phi-accrual
failure detector, SURVEY C41, and of the cluster singleton's leader choice, C44).

Every rank bumps a heartbeat counter ``hb/<rank>`` in the c10d store from a background
thread -- only while ``health()`` holds: a pipelined sharded rank gates it on its stepper
(``Frontend.healthy``: no failed engine, no GPU wait stuck past a deadline), so a wedged
GPU or a dead engine stops the beat even though the process lives.  ``suspects()``
reports ranks whose counter has not moved for ``timeout_s``.  ``agree_dead`` makes the
survivors converge: each publishes its suspicion set and the dead set is the union of
what the survivors report (a rank one survivor cannot reach would break every
collective), so all survivors re-home the same queues.  The leader (singleton duties: admin REST, store compaction) is the lowest
live rank.  The store must outlive any rank (launcher-hosted, parallel/launch.py).
"""

import threading
import time


class Membership:
    def __init__(self, store, rank, world, interval_s=0.2, timeout_s=2.0, health=None):
        self.store, self.rank, self.world = store, rank, world
        self.interval_s, self.timeout_s = interval_s, timeout_s
        self.health = health     # () -> bool: beat only while this rank makes progress
        self.live = set(range(world))
        self._seen = {r: (-1, time.monotonic()) for r in range(world)}
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._beat, name=f"hb-{rank}", daemon=True)
        self._t.start()

    def _beat(self):
        while not self._stop.is_set():
            try:
                if self.health is None or self.health():
                    self.store.add(f"hb/{self.rank}", 1)
            except Exception:   # store gone: the node is shutting down
                return
            self._stop.wait(self.interval_s)

    def stop(self):
        self._stop.set()
        if self._t.is_alive() and self._t is not threading.current_thread():
            self._t.join(timeout=5 * self.interval_s + 1.0)

    def suspects(self):
        now = time.monotonic()
        out = set()
        for r in self.live:
            if r == self.rank:
                continue
            v = self.store.add(f"hb/{r}", 0)
            last, t = self._seen[r]
            if v != last:
                self._seen[r] = (v, now)
            elif now - t > self.timeout_s:
                out.add(r)
        return out

    def wait_suspects(self, max_wait_s=None):
        """Block until some live peer is suspected (after a failed collective)."""
        end = time.monotonic() + (max_wait_s if max_wait_s is not None else 3 * self.timeout_s)
        while time.monotonic() < end:
            s = self.suspects()
            if s:
                return s
            time.sleep(self.interval_s)
        return set()

    def agree_dead(self, suspects, epoch):
        """Survivors publish their suspicions; the agreed dead set is the union of what
        the survivors see (a rank suspected by a survivor that is itself alive is dead
        to at least one peer, which is enough to break collectives)."""
        key = f"suspect/{epoch}/{self.rank}"
        self.store.set(key, ",".join(map(str, sorted(suspects))))
        cand = sorted(self.live - set(suspects))
        views = {}
        deadline = time.monotonic() + 5 * self.timeout_s
        while time.monotonic() < deadline:
            for r in cand:
                if r in views:
                    continue
                if self.store.check([f"suspect/{epoch}/{r}"]):
                    v = self.store.get(f"suspect/{epoch}/{r}").decode()
                    views[r] = set(int(x) for x in v.split(",") if x)
            if len(views) == len(cand):
                break
            time.sleep(self.interval_s / 2)
        dead = set(suspects)
        for r, v in views.items():
            dead |= v
        dead |= set(cand) - set(views)   # silent candidates are dead too
        dead.discard(self.rank)
        self.live -= dead
        return dead

    @property
    def leader(self):
        return min(self.live)
