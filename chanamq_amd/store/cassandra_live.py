"""Live Cassandra backend: the store's rows written through to a Cassandra keyspace while
the broker runs (the reference's CassandraOpService, chana-mq-server/src/main/scala/chana/mq/
amqp/server/store/cassandra/CassandraOpService.scala:70-86 prepared statements, 395-417
insertMessage / insertQueueMsg, 753-755 deletes).

The reference writes every row change to Cassandra from the entity that made it and waits
for nothing but the driver.  Here the embedded WAL store stays the broker's durable store
(its group commit gates publisher confirms), and ``CassandraMirror`` is its write-behind to
the cluster: the store marks the key of every row it changes (``Store.set_mirror``), the
mirror thread takes the marked keys every ``interval_s`` (``Store.mirror_take``), reads
each row's current state back and writes it with prepared INSERT / DELETE statements in
unlogged batches over the driverless CQL v4 client (``cql_native.CqlClient``):

* a row that exists now is upserted, a row that is gone is deleted -- so repeated changes
  to one row between two takes cost one write, and a message published and acked within
  one interval never reaches the cluster (as the store's own group delay keeps quickly
  acked bodies off the disk);
* range / whole-queue changes (``consumedQueueMessages``, queue deletes) mark the queue's
  partition: the mirror deletes the partition and writes its current rows;
* an exchange's bindings are rewritten as one partition (``binds`` is keyed by exchange).

The cluster therefore converges on the store's rows within about one interval plus the
write time; ``flush()`` waits for that.  ``cql_native.pull`` restores a store from the
keyspace (what the reference's recovery reads).  Errors are counted and the keys kept for
the next round (a cluster outage delays the mirror, never the broker).
"""

import threading
import time

from .cql import SCHEMA, ddl
from .cql_native import ONE, CqlClient, CqlError, encode_value


def _insert(ks, t):
    cols = [c for c, _ in SCHEMA[t][0]]
    return f"INSERT INTO {ks}.{t} ({', '.join(cols)}) VALUES ({', '.join('?' * len(cols))})"


def _delete(ks, t, keys):
    return f"DELETE FROM {ks}.{t} WHERE " + " AND ".join(f"{k} = ?" for k in keys)


class CassandraMirror:
    """Write-behind of a native ``Store``'s rows to ``keyspace`` on a Cassandra cluster."""

    def __init__(self, store, host="127.0.0.1", port=9042, keyspace="chanamq", user=None, password=None,
                 interval_s=0.05, batch=128, max_keys=4096, consistency=ONE, replication=1, create=True,
                 initial_push=True):
        self.store, self.ks, self.consistency = store, keyspace, consistency
        self.interval_s, self.batch, self.max_keys = interval_s, batch, max_keys
        self._conn = dict(host=host, port=port, user=user, password=password)
        self._create, self._replication, self._initial = create, replication, initial_push
        self.client = None
        self._th = None
        self._stop = threading.Event()
        self._idle = threading.Event()
        self._retry = None          # keys of a round that failed: written again first
        self.stats = dict(rounds=0, upserts=0, deletes=0, batches=0, partitions=0, errors=0, last_error="",
                          lag_s=0.0)

    # ---- lifecycle
    def start(self):
        self.client = CqlClient(**self._conn)
        if self._create:
            for stmt in ddl(self.ks, self._replication).split(";"):
                stmt = stmt.strip()
                if not stmt or stmt.upper().startswith("USE "):
                    continue
                if stmt.upper().startswith("CREATE TABLE"):
                    stmt = stmt.replace("CREATE TABLE IF NOT EXISTS ", f"CREATE TABLE IF NOT EXISTS {self.ks}.", 1)
                self.client.query(stmt, consistency=self.consistency)
        # from here on every change is marked; the rows already in the store go out first
        self.store.set_mirror(True)
        if self._initial:
            from .cql_native import push
            push(self.store, self.client, self.ks, self._replication, consistency=self.consistency)
        self._th = threading.Thread(target=self._run, name="cmq-cassandra", daemon=True)
        self._th.start()
        return self

    def stop(self, flush_s=5.0):
        if self._th is None:
            return
        if flush_s:
            self.flush(flush_s)
        self._stop.set()
        self._th.join(timeout=10)
        self._th = None
        self.store.set_mirror(False)
        self.client.close()

    def flush(self, timeout_s=5.0):
        """Wait until every change made before this call is in the cluster (True) or the
        timeout passed (False)."""
        end = time.monotonic() + timeout_s
        # two idle rounds after the call: the first may have taken keys marked before it
        seen = 0
        while time.monotonic() < end:
            self._idle.clear()
            if not self._idle.wait(max(0.0, end - time.monotonic())):
                return False
            if self.store.mirror_pending() == 0 and self._retry is None:
                seen += 1
                if seen >= 2:
                    return True
        return False

    # ---- the mirror thread
    def _run(self):
        while not self._stop.is_set():
            t0 = time.monotonic()
            try:
                n = self.round()
            except (CqlError, OSError) as e:   # kept for the next round
                self.stats["errors"] += 1
                self.stats["last_error"] = repr(e)
                n = 0
                try:
                    self.client.close()
                    self.client = CqlClient(**self._conn)
                except (CqlError, OSError):
                    pass
            self.stats["lag_s"] = round(time.monotonic() - t0, 4)
            self._idle.set()
            if n == 0:
                self._stop.wait(self.interval_s)

    def round(self):
        """One take of the marked keys -> statements -> batches; returns the keys written."""
        keys = self._retry or self.store.mirror_take(self.max_keys)
        self._retry = keys
        stmts = self._statements(keys)
        for k in range(0, len(stmts), self.batch):
            self.client.batch(stmts[k:k + self.batch], self.consistency)
            self.stats["batches"] += 1
        self._retry = None
        self.stats["rounds"] += 1
        return sum(len(v) for v in keys.values())

    def _statements(self, keys):
        st, ks, out = self.store, self.ks, []

        def up(t, row):
            out.append((_insert(ks, t), [encode_value(row.get(c), ty) for c, ty in SCHEMA[t][0]]))
            self.stats["upserts"] += 1

        def rm(t, kv):
            out.append((_delete(ks, t, [k for k, _ in kv]),
                        [encode_value(v, dict(SCHEMA[t][0])[k]) for k, v in kv]))
            self.stats["deletes"] += 1

        for v in keys["vhosts"]:
            a = st.select_vhost(v)
            up("vhosts", dict(id=v, active=bool(a))) if a is not None else rm("vhosts", [("id", v)])
        for x in keys["xs"]:
            r = st.select_exchange(x)
            rm("binds", [("id", x)])   # the exchange's binding partition, rewritten whole
            self.stats["partitions"] += 1
            if r is None:
                rm("exchanges", [("id", x)])
                continue
            (tpe, durable, autodel, internal, args), binds = r
            up("exchanges", dict(id=x, tpe=tpe, durable=durable, autodel=autodel, internal=internal, args=dict(args)))
            for q, key, bargs in binds:
                up("binds", dict(id=x, queue=q, key=key, args=dict(bargs)))
        for m in keys["msgs"]:   # before the queue rows that reference them
            r = st.select_message(m)
            if r is None:
                rm("msgs", [("id", m)])
                continue
            _, ts, header, body, ex, rk, durable, refer = r
            up("msgs", dict(id=m, tstamp=ts, header=bytes(header), body=bytes(body), exchange=ex, routing=rk,
                            durable=durable, refer=refer))
        for q in keys["qmetas"]:
            r = st.select_queue_meta(q)
            if r is None:
                rm("queue_metas", [("id", q)])
            else:
                lconsumed, consumers, durable, ttl = r
                up("queue_metas", dict(id=q, lconsumed=lconsumed, consumers=set(consumers), durable=durable, ttl=ttl))
        for q in keys["qparts"]:
            rm("queues", [("id", q)])
            rm("queue_unacks", [("id", q)])
            self.stats["partitions"] += 1
            r = st.select_queue(q)
            if r is not None:
                _, msgs, unacks = r
                for o, mid, size in msgs:
                    up("queues", dict(id=q, offset=o, msgid=mid, size=size))
                for o, mid, size in unacks:
                    up("queue_unacks", dict(id=q, offset=o, msgid=mid, size=size))
        for q, off in keys["qmsgs"]:
            r = st.select_queue_msg(q, off)
            if r is None:
                rm("queues", [("id", q), ("offset", off)])
            else:
                up("queues", dict(id=q, offset=r[0], msgid=r[1], size=r[2]))
        for q, mid in keys["qunacks"]:
            r = st.select_queue_unack(q, mid)
            if r is None:
                rm("queue_unacks", [("id", q), ("msgid", mid)])
            else:
                up("queue_unacks", dict(id=q, offset=r[0], msgid=r[1], size=r[2]))
        for q in keys["deleted"]:
            for t in ("queues_deleted", "queue_unacks_deleted", "queue_metas_deleted"):
                rm(t, [("id", q)])
            self.stats["partitions"] += 1
            meta, msgs, unacks = st.select_deleted_queue(q)
            if meta is not None:
                lconsumed, ncons, durable = meta
                up("queue_metas_deleted", dict(id=q, lconsumed=lconsumed, nconsumer=ncons, durable=durable))
            for o, mid, size in msgs:
                up("queues_deleted", dict(id=q, offset=o, msgid=mid, size=size))
            for o, mid, size in unacks:
                up("queue_unacks_deleted", dict(id=q, offset=o, msgid=mid, size=size))
        return out


__all__ = ["CassandraMirror"]
