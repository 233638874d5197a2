"""Durable store API (SURVEY §2 store layer; reference: chana-mq-server/.../store/cassandra/
CassandraOpService.scala and create-cassantra.cql).

The reference persists to Cassandra.  Here the same tables (msgs, queues, queue_unacks,
queue_metas, exchanges, binds, vhosts and their *_deleted copies) live in an embedded
store: in-memory tables rebuilt at open from a CRC-checked write-ahead log, one ``sync``
(group commit, fsync) per step that carries publisher confirms (csrc/core/store.cpp).
The GPU data plane writes to it through ``engine/persistence.py`` (Python rows) or the
native ``PersistWorker`` (csrc/core/persist.cpp, write-behind with group-commit
coalescing); a sharded broker keeps one store per rank (``rank_dir``) and survivors adopt a
dead rank's durable queues from its directory (``GpuPersistence.adopt``).
"""

import os

TABLES = ("msgs", "queues", "queue_unacks", "queue_metas", "exchanges", "binds", "vhosts",
          "queues_deleted", "queue_unacks_deleted", "queue_metas_deleted")


def _core():
    from ..broker import load
    return load()


def open_store(path, fsync=True):
    """Open (creating the directory) the store at ``path``; ``path=""`` is memory only.
    Replays the WAL and truncates a torn tail (a crash mid-append)."""
    if path:
        os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
    st = _core().Store()
    st.open(path, bool(fsync))
    return st


def rank_dir(root, rank):
    """A sharded broker's per-rank store directory."""
    return os.path.join(root, f"rank{int(rank)}")


def summary(store):
    """Row counts of every table (admin / tests)."""
    return {t: store.row_count(t) for t in TABLES}


def persist_worker(store):
    """The native write-behind worker over ``store`` (started by the caller)."""
    return _core().PersistWorker(store)


__all__ = ["TABLES", "open_store", "rank_dir", "summary", "persist_worker"]
