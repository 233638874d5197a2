"""Queue -> rank ownership for the sharded data plane.

The reference spreads queue entities over cluster nodes with Akka cluster sharding
(chana-mq-server/.../engine/QueueEntity.scala, Cluster.scala: ShardRegion with a hash
extractor) and re-homes them when a node leaves.  Here a rank is one MI355X (one
process), queues are owned by exactly one rank, and ownership is decided by rendezvous
(highest-random-weight) hashing over the live ranks: removing a rank moves only the
queues it owned, and every rank computes the same answer without coordination.
Explicit placement (``place``) overrides the hash, like RabbitMQ's queue-master locator,
and is what benchmarks use for an exactly balanced layout.
"""

from ..engine.control import entity_id
from ..engine.layout import fnv1a64

_M64 = (1 << 64) - 1


def _mix(x):
    """splitmix64 finaliser: spreads fnv1a64 output before the max-weight comparison."""
    x = (x + 0x9E3779B97F4A7C15) & _M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


class ShardMap:
    def __init__(self, world, live=None, placement=None):
        if world < 1:
            raise ValueError("world must be >= 1")
        self.world = world
        self.live = sorted(set(range(world) if live is None else live))
        self.placement = dict(placement or {})   # entity id -> rank

    def weight(self, rank, eid):
        return _mix(fnv1a64(eid.encode()) ^ ((rank + 1) * 0xD1B54A32D192ED03 & _M64))

    def owner_of(self, eid):
        r = self.placement.get(eid)
        if r is not None and r in self.live:
            return r
        return max(self.live, key=lambda k: (self.weight(k, eid), -k))

    def owner(self, vhost, name):
        return self.owner_of(entity_id(vhost, name))

    def place(self, vhost, name, rank):
        if not 0 <= rank < self.world:
            raise ValueError(f"rank {rank} out of range")
        self.placement[entity_id(vhost, name)] = rank

    def fail(self, rank):
        """Mark ``rank`` dead; returns the explicit placements that moved."""
        if rank in self.live:
            self.live.remove(rank)
        if not self.live:
            raise RuntimeError("no live ranks left")
        return [e for e, r in self.placement.items() if r == rank]

    def join(self, rank):
        if rank not in self.live:
            self.live = sorted(self.live + [rank])
