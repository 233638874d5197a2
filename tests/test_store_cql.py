"""Cassandra interop of the embedded store (chanamq_amd/store/cql.py): DDL for the
reference's tables, CQL INSERT export, and a CSV round trip (cqlsh COPY format) that
reproduces every row.  No Cassandra here: parity with a live cluster is unpinned; the
DDL is checked for the tables / keys the reference's keyspace declares."""

from chanamq_amd.store import open_store, summary
from chanamq_amd.store.cql import ddl, export_cql, export_csv, import_csv, rows


def _fill(st):
    st.insert_vhost("AMQ.DEFAULT", True)
    st.insert_exchange("AMQ.DEFAULT-_.x", "topic", True, False, False, {"alternate-exchange": "ae"})
    st.insert_bind("AMQ.DEFAULT-_.x", "AMQ.DEFAULT-_.q", "a.*", {})
    st.insert_queue_meta("AMQ.DEFAULT-_.q", -1, {"c1", "it's"}, True, 5000)
    for i in range(5):
        st.insert_message(100 + i, 1700000000000 + i, b"\0\0" + bytes(8) + b"\x10\x00\x02", b"body'%d\n" % i,
                          "x", "a.b", True, 1, 0)
        st.insert_queue_msg("AMQ.DEFAULT-_.q", i, 100 + i, 7, 0)
    st.insert_queue_unack("AMQ.DEFAULT-_.q", 9, 104, 7)
    st.sync()


def test_ddl_declares_the_reference_tables():
    text = ddl()
    for t in ("msgs", "queues", "queue_unacks", "queue_metas", "exchanges", "binds", "vhosts"):
        assert f"CREATE TABLE IF NOT EXISTS {t} (" in text
    assert "PRIMARY KEY ((id), offset)" in text and "CLUSTERING ORDER BY (offset ASC)" in text
    assert "PRIMARY KEY ((id), queue, key)" in text
    assert "consumers set<text>" in text and "args map<text, text>" in text


def test_cql_export_and_csv_round_trip(tmp_path):
    st = open_store(str(tmp_path / "a"), fsync=False)
    _fill(st)
    n = export_cql(st, str(tmp_path / "dump.cql"))
    assert n["msgs"] == 5 and n["queues"] == 5 and n["queue_unacks"] == 1
    text = (tmp_path / "dump.cql").read_text()
    assert "INSERT INTO msgs (id, tstamp, header, body, exchange, routing, durable, refer) VALUES (100," in text
    assert "{'c1', 'it''s'}" in text and "0x626f6479" in text
    export_csv(st, str(tmp_path / "csv"))
    before = rows(st)
    st.close()
    st2 = open_store(str(tmp_path / "b"), fsync=False)
    import_csv(st2, str(tmp_path / "csv"))
    after = rows(st2)
    for t in before:
        key = lambda r: sorted((k, repr(v)) for k, v in r.items())
        assert sorted(map(key, before[t])) == sorted(map(key, after[t])), t
    assert summary(st2)["msgs"] == 5
    st2.close()


def test_deleted_tables_ddl_export_and_round_trip(tmp_path):
    """queues_deleted / queue_metas_deleted / queue_unacks_deleted (create-cassantra.cql:48-74):
    pendingDeleteQueue copies a queue's rows there; DDL, CQL export and the CSV round trip
    carry them, and a compaction keeps them."""
    text = ddl()
    for t in ("queues_deleted", "queue_metas_deleted", "queue_unacks_deleted"):
        assert f"CREATE TABLE IF NOT EXISTS {t} (" in text
    assert "nconsumer int" in text
    st = open_store(str(tmp_path / "a"), fsync=False)
    _fill(st)
    st.pending_delete_queue("AMQ.DEFAULT-_.q")
    st.sync()
    assert summary(st)["queue_metas_deleted"] == 1
    assert summary(st)["queues_deleted"] == 5 and summary(st)["queue_unacks_deleted"] == 1
    n = export_cql(st, str(tmp_path / "dump.cql"))
    assert n["queues_deleted"] == 5 and n["queue_metas_deleted"] == 1 and n["queue_unacks_deleted"] == 1
    assert "INSERT INTO queue_metas_deleted (id, lconsumed, nconsumer, durable) VALUES ('AMQ.DEFAULT-_.q', -1, 2, true);" \
        in (tmp_path / "dump.cql").read_text()
    export_csv(st, str(tmp_path / "csv"))
    before = rows(st)
    st.compact()
    assert rows(st) == before
    st.close()
    st2 = open_store(str(tmp_path / "b"), fsync=False)
    import_csv(st2, str(tmp_path / "csv"))
    after = rows(st2)
    for t in ("queues_deleted", "queue_metas_deleted", "queue_unacks_deleted"):
        assert sorted(map(repr, before[t])) == sorted(map(repr, after[t])), t
    st2.close()
    st3 = open_store(str(tmp_path / "b"), fsync=False)   # replayed from its WAL
    assert summary(st3)["queues_deleted"] == 5 and summary(st3)["queue_metas_deleted"] == 1
    st3.close()


def test_live_push_and_pull_over_the_native_protocol(tmp_path):
    """store -> (CQL native protocol v4: STARTUP + PasswordAuthenticator, DDL, batched
    prepared INSERTs) -> a CQL server -> SELECT back into a fresh store: every row of every
    table survives.  The server is tests/cql_fake_server.py (no Cassandra here; it decodes
    the values with its own codec from the reference schema), so parity with a real
    cluster stays unpinned."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from cql_fake_server import FakeCql

    from chanamq_amd.store.cql_native import CqlClient, CqlError, pull, push
    srv = FakeCql(user="cassandra", password="secret")
    try:
        try:
            CqlClient(port=srv.port, user="cassandra", password="wrong")
            raise AssertionError("bad credentials accepted")
        except CqlError:
            pass
        st = open_store(str(tmp_path / "a"), fsync=False)
        _fill(st)
        st.pending_delete_queue("AMQ.DEFAULT-_.q")
        st.insert_queue_meta("AMQ.DEFAULT-_.q2", 3, set(), False, 0)
        st.sync()
        before = rows(st)
        with CqlClient(port=srv.port, user="cassandra", password="secret") as cl:
            n = push(st, cl, keyspace="cmq", batch=4)
        st.close()
        assert n["msgs"] == 5 and n["queues_deleted"] == 5 and n["queue_metas"] == 1
        assert any(s.startswith("CREATE KEYSPACE IF NOT EXISTS cmq") for s in srv.statements)
        assert len(srv.tables[("cmq", "msgs")]) == 5
        st2 = open_store(str(tmp_path / "b"), fsync=False)
        with CqlClient(port=srv.port, user="cassandra", password="secret") as cl:
            got = pull(cl, st2, keyspace="cmq")
        assert got == n
        after = rows(st2)
        for t in before:
            key = lambda r: sorted((k, repr(sorted(v) if isinstance(v, (set, frozenset)) else v)) for k, v in r.items())
            assert sorted(map(key, before[t])) == sorted(map(key, after[t])), t
        st2.close()
    finally:
        srv.close()
