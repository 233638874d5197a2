"""Bounded store: background WAL compaction (csrc/core/store.cpp compact_run) while group
commits keep appending.  The reference's Cassandra reclaims deleted rows itself
(CassandraOpService.scala:395-417 insert + delete paths); the embedded WAL must not grow
with total history (VERDICT r2 "store reclamation")."""

import os
import threading

from chanamq_amd.store import open_store, summary
from chanamq_amd.store.cql import rows


def _wal(d):
    return os.path.getsize(os.path.join(d, "chanamq.wal"))


def test_auto_compaction_keeps_wal_bounded_and_replays(tmp_path):
    d = str(tmp_path / "s")
    st = open_store(d, fsync=False)
    st.set_auto_compact(2.0, 1 << 20)
    st.insert_vhost("AMQ.DEFAULT", True)
    st.insert_queue_meta("AMQ.DEFAULT-_.q", -1, set(), True, 0)
    body = os.urandom(4096)
    live = {}
    mid = 1
    # config-4 shape: publish (message + queue row), then ack (delete both) a little later
    for rnd in range(400):
        for _ in range(32):
            st.insert_message(mid, 1, b"\0" * 10, body, "x", "k", True, 1, 0)
            st.insert_queue_msg("AMQ.DEFAULT-_.q", mid, mid, len(body), 0)
            live[mid] = True
            mid += 1
        for m in sorted(live)[:-64]:   # keep 64 live, ack the rest
            st.delete_queue_msg("AMQ.DEFAULT-_.q", m)
            st.delete_message(m)
            del live[m]
        st.sync()
    st.wait_compaction()
    cs = st.compact_stats()
    total_written = 400 * 32 * (4096 + 200)
    assert cs["runs"] >= 1, cs
    assert st.wal_bytes() < total_written / 4, (st.wal_bytes(), total_written)
    assert _wal(d) == st.wal_bytes()
    before = rows(st)
    st.close()
    st2 = open_store(d, fsync=False)
    assert rows(st2) == before
    assert summary(st2)["msgs"] == 64 and summary(st2)["queues"] == 64
    st2.close()


def test_compaction_under_concurrent_commits(tmp_path):
    """A writer thread keeps inserting / deleting / updating while compactions run; the
    reopened store equals the live one (snapshot + tail replay is order-safe)."""
    d = str(tmp_path / "c")
    st = open_store(d, fsync=False)
    st.set_auto_compact(0.0, 0)   # manual compactions only, racing the writer
    st.insert_vhost("v", True)
    st.insert_queue_meta("v-_.q", -1, set(), True, 0)
    stop = threading.Event()
    err = []

    def writer():
        try:
            i = 0
            while not stop.is_set():
                i += 1
                st.insert_message(i, i, b"h" * 10, b"b" * (64 + i % 512), "x", "k", True, 1, 0)
                st.insert_queue_msg("v-_.q", i, i, 10, 0)
                if i % 3 == 0:
                    st.update_message_refer_count(i, 2)
                if i > 50:
                    st.delete_queue_msg("v-_.q", i - 50)
                    st.delete_message(i - 50)
                if i % 7 == 0:
                    st.insert_queue_unack("v-_.q", i, i, 10)
                if i % 11 == 0:
                    st.delete_queue_unack("v-_.q", i - 7)
                if i % 64 == 0:
                    st.sync()
        except Exception as e:   # pragma: no cover - reported below
            err.append(e)

    th = threading.Thread(target=writer)
    th.start()
    for _ in range(6):
        st.compact()
    stop.set()
    th.join()
    assert not err, err
    st.sync()
    before = rows(st)
    assert st.compact_stats()["runs"] == 6
    st.close()
    st2 = open_store(d, fsync=False)
    assert rows(st2) == before
    st2.close()


def test_background_compaction_failure_is_contained(tmp_path):
    """an error inside the background compaction thread (here the
    .compact file cannot be created, standing in for ENOSPC/EIO) must not escape the
    thread.  The store keeps appending, records the failure, backs off, and a later run
    succeeds once the cause is gone; the synchronous compact() still raises."""
    import pytest
    d = str(tmp_path / "f")
    st = open_store(d, fsync=False)
    os.mkdir(os.path.join(d, "chanamq.wal.compact"))   # open(O_CREAT|O_TRUNC) -> EISDIR
    st.set_auto_compact(1.5, 1 << 16)
    st.insert_vhost("v", True)
    st.insert_queue_meta("v-_.q", -1, set(), True, 0)
    body = b"z" * 2048
    for i in range(1, 400):
        st.insert_message(i, 1, b"h" * 10, body, "x", "k", True, 1, 0)
        st.delete_message(i)
        if i % 16 == 0:
            st.sync()
            st.wait_compaction()
    cs = st.compact_stats()
    assert cs["runs"] == 0 and cs["failures"] >= 1, cs
    assert "compact" in cs["last_error"]
    # failures back off: far fewer attempts than group commits
    assert cs["failures"] < 400 // 16, cs
    with pytest.raises(RuntimeError):
        st.compact()
    os.rmdir(os.path.join(d, "chanamq.wal.compact"))
    st.compact()
    assert st.compact_stats()["runs"] == 1
    st.insert_message(10_000, 1, b"h" * 10, body, "x", "k", True, 1, 0)
    st.sync()
    before = rows(st)
    st.close()
    st2 = open_store(d, fsync=False)
    assert rows(st2) == before
    st2.close()
