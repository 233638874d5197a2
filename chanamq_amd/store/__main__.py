"""Store tools: ``python -m chanamq_amd.store <command> STORE_DIR ...``

  ddl                      print the Cassandra DDL of the store's tables
  summary  DIR             row counts
  export   DIR --cql FILE  live rows as CQL INSERT statements (with the DDL)
  export   DIR --csv OUT   one CSV per table (cqlsh COPY ... FROM)
  import   DIR --csv IN    CSV rows (cqlsh COPY ... TO, or export --csv) into the store
  push     DIR --cassandra HOST:PORT [--user U --password P]
                           live rows into a Cassandra keyspace over the CQL native protocol
  pull     DIR --cassandra HOST:PORT [...]
                           a Cassandra keyspace's rows into the store
"""
import argparse
import json
import sys

from . import open_store, summary
from .cql import ddl, export_cql, export_csv, import_csv


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m chanamq_amd.store")
    ap.add_argument("command", choices=["ddl", "summary", "export", "import", "push", "pull"])
    ap.add_argument("dir", nargs="?", default="")
    ap.add_argument("--cql", default="")
    ap.add_argument("--csv", default="")
    ap.add_argument("--keyspace", default="chanamq")
    ap.add_argument("--cassandra", default="127.0.0.1:9042", help="push / pull: HOST:PORT")
    ap.add_argument("--user", default=None)
    ap.add_argument("--password", default=None)
    a = ap.parse_args(argv)
    if a.command == "ddl":
        sys.stdout.write(ddl(a.keyspace))
        return 0
    if not a.dir:
        ap.error("the store directory is required")
    st = open_store(a.dir, fsync=True)
    try:
        if a.command == "summary":
            out = summary(st)
        elif a.command in ("push", "pull"):
            from .cql_native import CqlClient, pull, push
            host, _, port = a.cassandra.rpartition(":")
            with CqlClient(host or "127.0.0.1", int(port), a.user, a.password) as cl:
                out = push(st, cl, a.keyspace) if a.command == "push" else pull(cl, st, a.keyspace)
        elif a.command == "export":
            if not (a.cql or a.csv):
                ap.error("export needs --cql FILE or --csv DIR")
            out = export_cql(st, a.cql, a.keyspace) if a.cql else export_csv(st, a.csv)
        else:
            if not a.csv:
                ap.error("import needs --csv DIR")
            out = import_csv(st, a.csv)
        print(json.dumps(out))
    finally:
        st.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
