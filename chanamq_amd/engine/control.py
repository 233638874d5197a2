"""Control-plane state shared by every data-plane implementation.

The reference keeps this state in sharded actors (VhostEntity / ExchangeEntity /
QueueEntity, chana-mq-server/.../entity/*.scala) and per-connection objects
(AMQConnection / AMQChannel / AMQConsumer, chana-mq-base/.../model/*.scala).
Here it is a plain, deterministic, replicated table set: every rank applies the
same control ops in the same order and the GPU data plane receives
dense device tables built from it.
"""

from dataclasses import dataclass, field

from ..protocol import constants as C

DEFAULT_VHOST = "AMQ.DEFAULT"   # SR/reference.conf:129
VHOST_SEPARATOR = "-_."          # SR/reference.conf:135


def normalize_vhost(v: str) -> str:
    """Connection.Open vhost normalisation (FrameStage.scala:853-893): leading '/'
    stripped, empty -> default id."""
    if v.startswith("/"):
        v = v[1:]
    return v or DEFAULT_VHOST


def entity_id(vhost: str, name: str) -> str:
    """Entity id used as the Cassandra key: vhost + "-_." + name, or name when the
    vhost is empty (chana-mq-server/.../package.scala:17-21)."""
    return name if vhost == "" else f"{vhost}{VHOST_SEPARATOR}{name}"


@dataclass
class Exchange:
    slot: int
    vhost: str
    name: str
    type: str
    durable: bool = False
    auto_delete: bool = False
    internal: bool = False
    arguments: dict = field(default_factory=dict)
    bindings: list = field(default_factory=list)   # [(queue_slot, key bytes)]


@dataclass
class Queue:
    slot: int
    vhost: str
    name: str
    durable: bool = False
    exclusive_owner: int = -1
    auto_delete: bool = False
    ttl_ms: int = 0
    capacity: int = 1 << 16
    ring_off: int = 0
    consumers: list = field(default_factory=list)  # consumer ids, in registration order
    owner: int = 0                                  # owning rank (sharded data plane)
    requested: int = 0                              # requested ring capacity (for re-homing)
    max_capacity: int = 0                           # ring growth limit (0 = the ring pool)


@dataclass
class Channel:
    conn: int
    ch: int
    local: int
    confirm: bool = False
    prefetch_count: int = 0
    prefetch_size: int = 0
    global_: bool = False
    flow: bool = True
    tx: bool = False            # Tx.Select: publishes / acks held by the host until Tx.Commit
    consumers: dict = field(default_factory=dict)  # tag -> consumer id


@dataclass
class Connection:
    conn: int
    vhost: str
    frame_max: int = 131072
    channels: dict = field(default_factory=dict)   # ch -> Channel
    paused: bool = False


@dataclass
class Consumer:
    cid: int
    conn: int
    ch: int
    queue: int
    tag: str
    no_ack: bool
    active: bool = True


class ControlError(Exception):
    def __init__(self, code, text, class_id=0, method_id=0):
        super().__init__(f"{code} {text}")
        self.code, self.text, self.class_id, self.method_id = code, text, class_id, method_id


class ControlState:
    STANDARD_EXCHANGES = (("", "direct"), ("amq.direct", "direct"), ("amq.fanout", "fanout"),
                          ("amq.topic", "topic"), ("amq.headers", "headers"), ("amq.match", "headers"))

    def __init__(self, c_max=1024, chpc=16, q_max=4096, x_max=1024, cons_max=16384,
                 hash_wildcard=True, ring_pool=1 << 26, default_queue_capacity=1 << 16,
                 world=1, rank=0, shard_map=None):
        self.c_max, self.chpc, self.q_max, self.x_max, self.cons_max = c_max, chpc, q_max, x_max, cons_max
        # sharded data plane: every rank holds the same exchanges/bindings/queue slots
        # (control ops are applied on all ranks in the same order); a queue's ring,
        # consumers and deliveries live only on its owner (parallel/shard.py)
        self.world, self.rank = world, rank
        if world > 1 and shard_map is None:
            from ..parallel.shard import ShardMap
            shard_map = ShardMap(world)
        self.shard_map = shard_map
        self.hash_wildcard = hash_wildcard
        self.ring_pool = ring_pool
        self.default_queue_capacity = default_queue_capacity
        self.vhosts = {}             # name -> id
        self.exchanges = {}          # (vhost, name) -> Exchange
        self.queues = {}             # (vhost, name) -> Queue
        self.queue_by_slot = {}
        self.exch_by_slot = {}
        self.conns = {}              # conn -> Connection
        self.consumers = {}          # cid -> Consumer
        self._free_x = list(range(x_max - 1, -1, -1))
        self._free_q = list(range(q_max - 1, -1, -1))
        self._free_cid = list(range(cons_max - 1, -1, -1))
        self._ring_top = 0
        self._ring_free = {}         # capacity -> [offsets]
        self.ensure_vhost(DEFAULT_VHOST)

    # ------------------------------------------------------------------ vhosts
    def ensure_vhost(self, name):
        if name not in self.vhosts:
            self.vhosts[name] = len(self.vhosts)
            for xn, xt in self.STANDARD_EXCHANGES:
                self.declare_exchange(name, xn, xt, durable=True, _sync=False)
            self.routing_changed()
        return self.vhosts[name]

    # ------------------------------------------------------------------ connections
    def open_connection(self, conn, vhost=DEFAULT_VHOST, frame_max=131072):
        if not 0 <= conn < self.c_max:
            raise ControlError(C.RESOURCE_ERROR, "connection slot out of range")
        self.ensure_vhost(vhost)
        self.conns[conn] = Connection(conn, vhost, frame_max)
        self.connection_changed(conn)
        return conn

    def close_connection(self, conn):
        c = self.conns.get(conn)
        if c is None:
            return
        for ch in list(c.channels):
            self.close_channel(conn, ch)
        for q in [q for q in self.queues.values() if q.exclusive_owner == conn]:
            self.delete_queue(q.vhost, q.name)
        del self.conns[conn]
        self.connection_changed(conn)

    def open_channel(self, conn, ch):
        c = self.conns[conn]
        if ch in c.channels:
            raise ControlError(C.CHANNEL_ERROR, "channel already open", 20, 10)
        used = {x.local for x in c.channels.values()}
        free = [i for i in range(self.chpc) if i not in used]
        if not free:
            raise ControlError(C.RESOURCE_ERROR, "too many channels on the GPU path", 20, 10)
        chan = Channel(conn, ch, free[0])
        c.channels[ch] = chan
        self.channel_opened(chan)
        return self.chslot(conn, ch)

    def close_channel(self, conn, ch):
        c = self.conns.get(conn)
        if c is None or ch not in c.channels:
            return
        chan = c.channels[ch]
        for tag in list(chan.consumers):
            self.cancel(conn, ch, tag)
        self.channel_closing(chan)
        del c.channels[ch]

    def chslot(self, conn, ch):
        return conn * self.chpc + self.conns[conn].channels[ch].local

    def channel(self, conn, ch):
        return self.conns[conn].channels[ch]

    def confirm_select(self, conn, ch):
        self.channel(conn, ch).confirm = True
        self.channel_changed(conn, ch)

    def tx_select(self, conn, ch):
        self.channel(conn, ch).tx = True
        self.channel_changed(conn, ch)

    def qos(self, conn, ch, prefetch_count, prefetch_size=0, global_=False):
        chan = self.channel(conn, ch)
        chan.prefetch_count, chan.prefetch_size, chan.global_ = prefetch_count, prefetch_size, global_
        self.channel_changed(conn, ch)

    def flow(self, conn, ch, active):
        self.channel(conn, ch).flow = bool(active)
        self.channel_changed(conn, ch)

    # ------------------------------------------------------------------ exchanges
    def declare_exchange(self, vhost, name, type_="direct", durable=False, auto_delete=False,
                         internal=False, arguments=None, passive=False, _sync=True):
        key = (vhost, name)
        x = self.exchanges.get(key)
        if x is not None:
            return x.slot
        if passive:
            raise ControlError(C.NOT_FOUND, f"no exchange '{name}' in vhost '{vhost}'", 40, 10)
        if type_ not in C.EXCHANGE_TYPES:
            raise ControlError(C.COMMAND_INVALID, f"unknown exchange type '{type_}'", 40, 10)
        if not self._free_x:
            raise ControlError(C.RESOURCE_ERROR, "exchange table full", 40, 10)
        slot = self._free_x.pop()
        x = Exchange(slot, vhost, name, type_, durable, auto_delete, internal, dict(arguments or {}))
        self.exchanges[key] = x
        self.exch_by_slot[slot] = x
        if name == "":  # default exchange: implicit binding of every queue by name
            for q in self.queues.values():
                if q.vhost == vhost:
                    x.bindings.append((q.slot, q.name.encode()))
        if _sync:
            self.routing_changed()
        return slot

    def delete_exchange(self, vhost, name, if_unused=False):
        x = self.exchanges.get((vhost, name))
        if x is None:
            raise ControlError(C.NOT_FOUND, f"no exchange '{name}' in vhost '{vhost}'", 40, 20)
        if if_unused and x.bindings:
            raise ControlError(C.PRECONDITION_FAILED, f"exchange '{name}' in use", 40, 20)
        del self.exchanges[(vhost, name)]
        del self.exch_by_slot[x.slot]
        self._free_x.append(x.slot)
        self.routing_changed()

    # ------------------------------------------------------------------ queues
    def _ring_alloc(self, cap):
        lst = self._ring_free.get(cap)
        if lst:
            return lst.pop()
        if self._ring_top + cap > self.ring_pool:
            raise ControlError(C.RESOURCE_ERROR, "ring pool exhausted")
        off = self._ring_top
        self._ring_top += cap
        return off

    def declare_queue(self, vhost, name, durable=False, exclusive_owner=-1, auto_delete=False,
                      ttl_ms=0, capacity=None, passive=False, max_capacity=0):
        key = (vhost, name)
        q = self.queues.get(key)
        if q is not None:
            return q.slot
        if passive:
            raise ControlError(C.NOT_FOUND, f"no queue '{name}' in vhost '{vhost}'", 50, 10)
        if not self._free_q:
            raise ControlError(C.RESOURCE_ERROR, "queue table full", 50, 10)
        capacity = capacity or self.default_queue_capacity
        owner = self.shard_map.owner(vhost, name) if self.world > 1 else self.rank
        cap = 1
        while cap < capacity and owner == self.rank:   # remote queues hold no ring here
            cap <<= 1
        slot = self._free_q.pop()
        q = Queue(slot, vhost, name, durable, exclusive_owner, auto_delete, ttl_ms, cap,
                  self._ring_alloc(cap), owner=owner, requested=capacity, max_capacity=max_capacity)
        self.queues[key] = q
        self.queue_by_slot[slot] = q
        dx = self.exchanges.get((vhost, ""))
        if dx is not None:
            dx.bindings.append((slot, name.encode()))
        self.queue_declared(q)
        self.routing_changed()
        return slot

    def grow_target(self, q, depth):
        """Ring capacity for a queue holding ``depth`` entries once it passed half its ring:
        doubled until the depth is at most half of it, within max_capacity and the pool
        (None = no growth).  QueueEntity.scala:271-316 is an unbounded Vector; here the
        bound is the HBM ring pool (16 B per entry), and the body-log watermark pushes back
        on publishers long before it."""
        cap = q.capacity
        limit = q.max_capacity or self.ring_pool
        new = cap
        while depth * 2 > new and new * 2 <= limit:
            new *= 2
        return new if new > cap else None

    def regrow_ring(self, q, new_cap):
        """Allocate a ring of ``new_cap`` for queue ``q`` and release the old one; returns
        (old offset, old capacity) or None when the pool has no room."""
        try:
            off = self._ring_alloc(new_cap)
        except ControlError:
            return None
        old = (q.ring_off, q.capacity)
        self._ring_free.setdefault(q.capacity, []).append(q.ring_off)
        q.ring_off, q.capacity = off, new_cap
        return old

    def delete_queue(self, vhost, name):
        q = self.queues.pop((vhost, name), None)
        if q is None:
            raise ControlError(C.NOT_FOUND, f"no queue '{name}' in vhost '{vhost}'", 50, 40)
        for cid in list(q.consumers):
            c = self.consumers[cid]
            chan = self.conns[c.conn].channels.get(c.ch)
            if chan is not None:
                chan.consumers.pop(c.tag, None)
            self._drop_consumer(cid)
        for x in self.exchanges.values():   # QueueDeleted broadcast (ExchangeEntity.scala:191-193)
            x.bindings = [(s, k) for s, k in x.bindings if s != q.slot]
        del self.queue_by_slot[q.slot]
        # a freed slot is reused last (FIFO), not next: a request still naming the old slot
        # (a Basic.Get staged for a step) must not land on a queue declared right after
        self._free_q.insert(0, q.slot)
        self._ring_free.setdefault(q.capacity, []).append(q.ring_off)
        self.queue_deleted(q)
        self.routing_changed()

    def set_queue_owner(self, slot, owner):
        """Move queue ``slot`` to rank ``owner`` (failover re-homing, placement).  The new
        owner allocates a fresh ring; the old owner's ring is released (it must be the
        dead rank's, or empty).  Applied identically on every rank (control log)."""
        q = self.queue_by_slot[slot]
        if q.owner == owner:
            return owner
        if q.owner == self.rank:
            for cid in list(q.consumers):
                c = self.consumers[cid]
                self.channel(c.conn, c.ch).consumers.pop(c.tag, None)
                self._drop_consumer(cid)
        self._ring_free.setdefault(q.capacity, []).append(q.ring_off)
        cap = 1
        while cap < (q.requested or self.default_queue_capacity) and owner == self.rank:
            cap <<= 1
        q.owner, q.capacity, q.ring_off = owner, cap, self._ring_alloc(cap)
        self.queue_declared(q)
        self.routing_changed()
        return owner

    def rehome(self, dead):
        """Re-home every queue owned by the ``dead`` ranks (ShardMap already updated)."""
        moved = []
        for q in sorted(self.queue_by_slot.values(), key=lambda x: x.slot):
            if q.owner in dead:
                self.set_queue_owner(q.slot, self.shard_map.owner(q.vhost, q.name))
                moved.append(q.name)
        return moved

    def bind(self, vhost, queue, exchange, key):
        x = self.exchanges.get((vhost, exchange))
        q = self.queues.get((vhost, queue))
        if x is None:
            raise ControlError(C.NOT_FOUND, f"no exchange '{exchange}' in vhost '{vhost}'", 50, 20)
        if q is None:
            raise ControlError(C.NOT_FOUND, f"no queue '{queue}' in vhost '{vhost}'", 50, 20)
        if exchange == "":
            raise ControlError(C.ACCESS_REFUSED, "operation not permitted on the default exchange", 50, 20)
        kb = key.encode() if isinstance(key, str) else bytes(key)
        if (q.slot, kb) not in x.bindings:
            x.bindings.append((q.slot, kb))
            self.routing_changed()

    def route_host(self, x, key):
        """Queue slots a publish with routing key ``key`` (bytes) reaches through exchange
        ``x``, from the replicated binding table (what the device routes; headers routes as
        topic).  Host-side routing for host-assembled large publishes."""
        from ..models.matcher import topic_match
        if x.type == "fanout":
            return sorted({s for s, _ in x.bindings})
        if x.type == "direct":
            return sorted({s for s, k in x.bindings if k == key})
        ks = key.decode(errors="replace")
        return sorted({s for s, k in x.bindings if topic_match(k.decode(errors="replace"), ks, self.hash_wildcard)})

    def unbind(self, vhost, queue, exchange, key):
        x = self.exchanges.get((vhost, exchange))
        q = self.queues.get((vhost, queue))
        if x is None or q is None:
            raise ControlError(C.NOT_FOUND, "no such binding", 50, 50)
        kb = key.encode() if isinstance(key, str) else bytes(key)
        if (q.slot, kb) in x.bindings:
            x.bindings.remove((q.slot, kb))
            self.routing_changed()

    # ------------------------------------------------------------------ consumers
    def consume(self, conn, ch, queue_vhost, queue, tag, no_ack=False):
        q = self.queues.get((queue_vhost, queue))
        if q is None:
            raise ControlError(C.NOT_FOUND, f"no queue '{queue}'", 60, 20)
        if q.owner != self.rank:
            # consumers attach on the owning rank (the front end places the connection there)
            raise ControlError(C.NOT_ALLOWED, f"queue '{queue}' is served by rank {q.owner}", 60, 20)
        chan = self.channel(conn, ch)
        if tag in chan.consumers:
            raise ControlError(C.NOT_ALLOWED, f"consumer tag '{tag}' in use", 60, 20)
        if not self._free_cid:
            raise ControlError(C.RESOURCE_ERROR, "consumer table full", 60, 20)
        cid = self._free_cid.pop()
        self.consumers[cid] = Consumer(cid, conn, ch, q.slot, tag, no_ack)
        chan.consumers[tag] = cid
        q.consumers.append(cid)
        self.consumers_changed(q, cid)
        return cid

    def cancel(self, conn, ch, tag):
        chan = self.channel(conn, ch)
        cid = chan.consumers.pop(tag, None)
        if cid is None:
            return None
        self._drop_consumer(cid)
        return cid

    def _drop_consumer(self, cid):
        c = self.consumers.pop(cid)
        q = self.queue_by_slot.get(c.queue)
        if q is not None and cid in q.consumers:
            q.consumers.remove(cid)
            self.consumers_changed(q, cid, removed=True)
        self._free_cid.append(cid)

    # ------------------------------------------------------------------ hooks (overridden)
    def routing_changed(self): ...
    def connection_changed(self, conn): ...
    def channel_opened(self, chan): ...
    def channel_changed(self, conn, ch): ...
    def channel_closing(self, chan): ...
    def queue_declared(self, q): ...
    def queue_deleted(self, q): ...
    def consumers_changed(self, q, cid, removed=False): ...
