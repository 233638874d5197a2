"""Cassandra interop for the embedded store (reference: the CQL keyspace the reference
broker creates and CassandraOpService.scala writes).

The broker keeps the reference's tables in an embedded WAL store; this module moves
rows to and from a real Cassandra deployment:

* ``ddl()``        — CREATE KEYSPACE / TABLE statements for the tables the store holds
                     (same names, column types, primary keys and clustering order)
* ``export_cql``   — the store's live rows as CQL INSERT statements (``cqlsh -f``)
* ``export_csv``   — one CSV per table in ``cqlsh COPY <table> FROM`` format
* ``import_csv``   — the reverse: rows exported from Cassandra (``COPY ... TO``) or by
                     ``export_csv`` into a store

Blobs are hex (``0x…`` in CQL, bare hex in CSV), sets / maps use CQL collection
literals.  Per-row TTLs are not carried (rows are exported as live at export time).
"""

import csv
import os

# table -> ([(column, cql type)], partition key, clustering columns)
SCHEMA = {
    "msgs": ([("id", "bigint"), ("tstamp", "bigint"), ("header", "blob"), ("body", "blob"), ("exchange", "text"),
              ("routing", "text"), ("durable", "boolean"), ("refer", "int")], ["id"], []),
    "queues": ([("id", "text"), ("offset", "bigint"), ("msgid", "bigint"), ("size", "int")], ["id"], ["offset"]),
    "queue_unacks": ([("id", "text"), ("offset", "bigint"), ("msgid", "bigint"), ("size", "int")], ["id"], ["msgid"]),
    "queue_metas": ([("id", "text"), ("lconsumed", "bigint"), ("consumers", "set<text>"), ("durable", "boolean"),
                     ("ttl", "bigint")], ["id"], []),
    "exchanges": ([("id", "text"), ("tpe", "text"), ("durable", "boolean"), ("autodel", "boolean"),
                   ("internal", "boolean"), ("args", "map<text, text>")], ["id"], []),
    "binds": ([("id", "text"), ("queue", "text"), ("key", "text"), ("args", "map<text, text>")], ["id"],
              ["queue", "key"]),
    "vhosts": ([("id", "text"), ("active", "boolean")], ["id"], []),
    # rows of queues removed by pendingDeleteQueue (create-cassantra.cql:48-74,
    # CassandraOpService.scala:561-604; nconsumer is an int, SURVEY A.Q22)
    "queues_deleted": ([("id", "text"), ("offset", "bigint"), ("msgid", "bigint"), ("size", "int")], ["id"],
                       ["offset"]),
    "queue_metas_deleted": ([("id", "text"), ("lconsumed", "bigint"), ("nconsumer", "int"), ("durable", "boolean")],
                            ["id"], []),
    "queue_unacks_deleted": ([("id", "text"), ("offset", "bigint"), ("msgid", "bigint"), ("size", "int")], ["id"],
                             ["msgid"]),
}
ORDER = ["vhosts", "exchanges", "binds", "queue_metas", "msgs", "queues", "queue_unacks", "queues_deleted",
         "queue_metas_deleted", "queue_unacks_deleted"]


def ddl(keyspace="chanamq", replication=1):
    out = [f"CREATE KEYSPACE IF NOT EXISTS {keyspace} WITH REPLICATION = "
           f"{{'class': 'SimpleStrategy', 'replication_factor': '{int(replication)}'}} AND DURABLE_WRITES = true;",
           f"USE {keyspace};"]
    for t in ORDER:
        cols, pk, ck = SCHEMA[t]
        body = ",\n".join(f"  {c} {ty}" for c, ty in cols)
        key = f"({', '.join(pk)})" + "".join(f", {c}" for c in ck)
        stmt = f"CREATE TABLE IF NOT EXISTS {t} (\n{body},\n  PRIMARY KEY ({key})\n)"
        if ck:
            stmt += " WITH CLUSTERING ORDER BY (" + ", ".join(f"{c} ASC" for c in ck) + ")"
        out.append(stmt + ";")
    return "\n\n".join(out) + "\n"


# ---------------------------------------------------------------------------- rows
def rows(store):
    """{table: [dict row]} of the store's live rows."""
    out = {t: [] for t in ORDER}
    for v in store.vhost_ids():
        out["vhosts"].append(dict(id=v, active=True))
    for xid in store.exchange_ids():
        r = store.select_exchange(xid)
        if r is None:
            continue
        (tpe, durable, autodel, internal, args), binds = r
        out["exchanges"].append(dict(id=xid, tpe=tpe, durable=durable, autodel=autodel, internal=internal,
                                     args=dict(args)))
        for q, key, bargs in binds:
            out["binds"].append(dict(id=xid, queue=q, key=key, args=dict(bargs)))
    for qid in store.queue_ids():
        r = store.select_queue(qid)
        if r is None:
            continue
        (lconsumed, consumers, durable, ttl), msgs, unacks = r
        out["queue_metas"].append(dict(id=qid, lconsumed=lconsumed, consumers=set(consumers), durable=durable,
                                       ttl=ttl))
        out["queues"] += [dict(id=qid, offset=o, msgid=m, size=s) for o, m, s in msgs]
        out["queue_unacks"] += [dict(id=qid, offset=o, msgid=m, size=s) for o, m, s in unacks]
    for qid in (store.deleted_queue_ids() if hasattr(store, "deleted_queue_ids") else ()):
        meta, msgs, unacks = store.select_deleted_queue(qid)
        if meta is not None:
            lconsumed, ncons, durable = meta
            out["queue_metas_deleted"].append(dict(id=qid, lconsumed=lconsumed, nconsumer=ncons, durable=durable))
        out["queues_deleted"] += [dict(id=qid, offset=o, msgid=m, size=s) for o, m, s in msgs]
        out["queue_unacks_deleted"] += [dict(id=qid, offset=o, msgid=m, size=s) for o, m, s in unacks]
    for mid in store.message_ids():
        m = store.select_message(mid)
        if m is None:
            continue
        _, ts, header, body, ex, rk, durable, refer = m
        out["msgs"].append(dict(id=mid, tstamp=ts, header=bytes(header), body=bytes(body), exchange=ex, routing=rk,
                                durable=durable, refer=refer))
    return out


def _q(s):
    return "'" + str(s).replace("'", "''") + "'"


def _lit(v, ty):
    if ty == "blob":
        return "0x" + bytes(v).hex()
    if ty == "text":
        return _q(v)
    if ty == "boolean":
        return "true" if v else "false"
    if ty.startswith("set"):
        return "{" + ", ".join(_q(x) for x in sorted(v)) + "}"
    if ty.startswith("map"):
        return "{" + ", ".join(f"{_q(k)}: {_q(x)}" for k, x in sorted(v.items())) + "}"
    return str(int(v))


def export_cql(store, path, keyspace="chanamq", with_ddl=True):
    """All live rows as INSERT statements (plus the DDL); returns rows written per table."""
    data = rows(store)
    n = {}
    with open(path, "w") as f:
        if with_ddl:
            f.write(ddl(keyspace))
            f.write("\n")
        else:
            f.write(f"USE {keyspace};\n")
        for t in ORDER:
            cols = SCHEMA[t][0]
            names = ", ".join(c for c, _ in cols)
            for r in data[t]:
                vals = ", ".join(_lit(r[c], ty) for c, ty in cols)
                f.write(f"INSERT INTO {t} ({names}) VALUES ({vals});\n")
            n[t] = len(data[t])
    return n


# ---------------------------------------------------------------------------- CSV (cqlsh COPY)
def _csv_val(v, ty):
    if ty == "blob":
        return "0x" + bytes(v).hex()
    if ty == "boolean":
        return "True" if v else "False"
    if ty.startswith("set"):
        return "{" + ", ".join(_q(x) for x in sorted(v)) + "}"
    if ty.startswith("map"):
        return "{" + ", ".join(f"{_q(k)}: {_q(x)}" for k, x in sorted(v.items())) + "}"
    return str(v)


def _parse_coll(s):
    """CQL collection literal ({'a', 'b'} or {'k': 'v'}) -> set / dict."""
    s = s.strip()
    if not s or s in ("{}", "null"):
        return None
    inner, items, cur, i, q = s[1:-1], [], "", 0, False
    while i < len(inner):
        ch = inner[i]
        if q:
            if ch == "'" and i + 1 < len(inner) and inner[i + 1] == "'":
                cur += "'"
                i += 2
                continue
            if ch == "'":
                q = False
            else:
                cur += ch
        elif ch == "'":
            q = True
        elif ch in ",:":
            items.append((cur, ch))
            cur = ""
        i += 1
    items.append((cur, ""))
    if any(sep == ":" for _, sep in items):
        vals = [x for x, _ in items]
        return {vals[k].strip(): vals[k + 1].strip() for k in range(0, len(vals) - 1, 2)}
    return {x.strip() for x, _ in items}


def _from_csv(v, ty):
    if ty == "blob":
        return bytes.fromhex(v[2:] if v.startswith("0x") else v)
    if ty == "boolean":
        return v.strip().lower() == "true"
    if ty.startswith("set"):
        return _parse_coll(v) or set()
    if ty.startswith("map"):
        return _parse_coll(v) or {}
    if ty == "text":
        return v
    return int(v)


def export_csv(store, out_dir):
    """One ``<table>.csv`` per table (header row = column names), loadable with
    ``COPY <table> (<columns>) FROM '<table>.csv' WITH HEADER = true``."""
    os.makedirs(out_dir, exist_ok=True)
    data = rows(store)
    n = {}
    for t in ORDER:
        cols = SCHEMA[t][0]
        with open(os.path.join(out_dir, f"{t}.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow([c for c, _ in cols])
            for r in data[t]:
                w.writerow([_csv_val(r[c], ty) for c, ty in cols])
        n[t] = len(data[t])
    return n


def import_csv(store, in_dir):
    """Rows from ``<table>.csv`` files (``COPY <table> TO ... WITH HEADER = true`` or
    ``export_csv``) into ``store``; tables without a file are skipped.  Commits."""
    n = {}
    for t in ORDER:
        p = os.path.join(in_dir, f"{t}.csv")
        if not os.path.exists(p):
            continue
        types = dict(SCHEMA[t][0])
        with open(p, newline="") as f:
            rd = csv.DictReader(f)
            k = 0
            for raw in rd:
                r = {c: _from_csv(v, types[c]) for c, v in raw.items() if c in types}
                _insert(store, t, r)
                k += 1
        n[t] = k
    store.sync()
    return n


def _insert(st, t, r):
    if t == "vhosts":
        st.insert_vhost(r["id"], bool(r.get("active", True)))
    elif t == "exchanges":
        st.insert_exchange(r["id"], r["tpe"], r["durable"], r["autodel"], r["internal"], r.get("args") or {})
    elif t == "binds":
        st.insert_bind(r["id"], r["queue"], r["key"], r.get("args") or {})
    elif t == "queue_metas":
        st.insert_queue_meta(r["id"], r["lconsumed"], set(r.get("consumers") or ()), r["durable"], r["ttl"])
    elif t == "msgs":
        st.insert_message(r["id"], r["tstamp"], r["header"], r["body"], r["exchange"], r["routing"], r["durable"],
                          r["refer"], 0)
    elif t == "queues":
        st.insert_queue_msg(r["id"], r["offset"], r["msgid"], r["size"], 0)
    elif t == "queue_unacks":
        st.insert_queue_unack(r["id"], r["offset"], r["msgid"], r["size"])
    elif t == "queues_deleted":
        st.insert_deleted_queue_msg(r["id"], r["offset"], r["msgid"], r["size"])
    elif t == "queue_metas_deleted":
        st.insert_deleted_queue_meta(r["id"], r["lconsumed"], r["nconsumer"], r["durable"])
    elif t == "queue_unacks_deleted":
        st.insert_deleted_queue_unack(r["id"], r["offset"], r["msgid"], r["size"])


__all__ = ["SCHEMA", "ORDER", "ddl", "rows", "export_cql", "export_csv", "import_csv"]
