"""``python -m chanamq_amd.server`` — the broker launcher (AMQPServer.scala:39-133).

  --config FILE        HOCON file layered over conf/reference.conf (like -Dconfig.file)
  --set key=value      override one key (repeatable)
  --stats-interval S   log the "published msgs" / "delivered msgs" counters every S seconds
                       (the lines chana-mq-test/perf/sum-published.sh scrapes)
  --data-plane host|gpu  host = native C++ broker (CPU data path, store, TLS);
                       gpu = the HIP data plane on --device behind server/gpu_broker.py
"""

import argparse
import json
import logging
import signal
import sys
import threading

from ..broker import load
from ..utils.config import Config
from .admin import AdminServer


def main(argv=None):
    ap = argparse.ArgumentParser(prog="chanamq_amd.server")
    ap.add_argument("--config", action="append", default=[])
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE")
    ap.add_argument("--stats-interval", type=float, default=10.0)
    ap.add_argument("--log-level", default="INFO")
    ap.add_argument("--data-plane", choices=["host", "gpu"], default="host")
    ap.add_argument("--device", type=int, default=None, help="GPU mode: device (default chana.mq.gpu.device)")
    ap.add_argument("--admin-port", type=int, default=None,
                    help="GPU mode: admin REST port (0 = any, -1 = off; default chana.mq.amqp.admin.port)")
    args = ap.parse_args(argv)
    logging.basicConfig(level=args.log_level, format="%(asctime)s:%(levelname)s %(threadName)s - %(message)s")
    log = logging.getLogger("chanamq")
    overrides = dict(kv.split("=", 1) for kv in args.set)
    cfg = Config.load(args.config, overrides)
    bc = cfg.broker_config()
    if args.data_plane == "gpu" or bool(cfg.get("chana.mq.gpu.enable", False)):
        return _main_gpu(args, bc, cfg, log)
    core = load()
    broker = core.Broker(bc)
    broker.start()
    log.info("AMQP listening on %s:%s%s", bc["host"], broker.port,
             f", AMQPS on {broker.tls_port}" if bc["tls_enable"] else "")
    admin = AdminServer(broker, int(cfg.get("chana.mq.amqp.admin.port"))).start()
    log.info("admin REST on 127.0.0.1:%d", admin.port)
    stop = threading.Event()
    for sig in (signal.SIGINT, signal.SIGTERM):
        signal.signal(sig, lambda *a: stop.set())
    last = {}
    while not stop.wait(args.stats_interval):
        s = json.loads(broker.stats_json())
        log.info("server published msgs: %d", s["published"] - last.get("published", 0))
        log.info("server delivered msgs: %d", s["delivered"] - last.get("delivered", 0))
        last = s
    admin.stop()
    broker.stop()
    return 0


def _main_gpu(args, bc, cfg, log):
    """GPU data plane behind the pipelined native front end, configured from
    ``chana.mq.gpu.*`` / ``chana.mq.store.*`` / ``chana.mq.flow.*`` / ``chana.mq.amqps.*``
    (AMQPServer.scala:52-106: store, AMQP + AMQPS listeners, admin REST)."""
    from ..engine.dataplane import GpuDataPlane
    from .gpu_broker import GpuBroker
    plane_kw, broker_kw = cfg.gpu_config()
    if args.device is not None:
        plane_kw["device"] = args.device
    core = load()
    store = None
    mirror = None
    if bc["data_dir"]:
        from ..store import open_store
        store = open_store(bc["data_dir"], bc["fsync"])
        mirror = _cassandra_live(cfg, store, log)
    plane = GpuDataPlane(**plane_kw)
    broker = GpuBroker(plane, host=bc["host"], port=bc["port"], heartbeat=bc["heartbeat"], frame_max=bc["frame_max"],
                       channel_max=bc["channel_max"] or 2047, store=store, **broker_kw).start()
    log.info("AMQP (GPU data plane, device %d, %s front end) listening on %s:%s; recovered %d messages",
             plane_kw["device"], broker.io, bc["host"], broker.port, broker.recovered)
    tls = None
    if bc["tls_enable"]:
        tls = core.TlsProxy(dict(host=bc["host"], port=bc["tls_port"], upstream_port=broker.port,
                                 cert=bc["tls_cert"], key=bc["tls_key"], p12=bc["tls_p12"],
                                 p12_password=bc["tls_p12_password"]))
        tls.start()
        log.info("AMQPS (TLS) on %s:%d -> the GPU front end", bc["host"], tls.port)
    broker.tls = tls
    admin_port = args.admin_port if args.admin_port is not None else int(cfg.get("chana.mq.amqp.admin.port"))
    admin = AdminServer(broker, admin_port).start() if admin_port >= 0 else None
    if admin is not None:
        log.info("admin REST on 127.0.0.1:%d", admin.port)
    stop = threading.Event()
    for sig in (signal.SIGINT, signal.SIGTERM):
        signal.signal(sig, lambda *a: stop.set())
    last = {}
    while not stop.wait(args.stats_interval):
        s = dict(broker.stats)
        log.info("server published msgs: %d", s["published"] - last.get("published", 0))
        log.info("server delivered msgs: %d", s["delivered"] - last.get("delivered", 0))
        last = s
    if admin is not None:
        admin.stop()
    if tls is not None:
        tls.stop()
    broker.stop()
    if mirror is not None:
        mirror.stop()
    if store is not None:
        store.close()
    return 0


def _cassandra_live(cfg, store, log):
    """``chana.mq.store.cassandra-live``: the store's rows written through to the
    ``chana.mq.cassandra.pass-through`` keyspace while the broker runs (the reference's
    CassandraOpService); ``cassandra-recover`` first fills an empty store from it."""
    if not bool(cfg.get("chana.mq.store.cassandra-live", False)):
        return None
    from ..store.cassandra_live import CassandraMirror
    from ..store.cql_native import CqlClient, pull
    hosts = cfg.get("chana.mq.cassandra.pass-through.hosts", ["localhost"])
    host = hosts[0] if isinstance(hosts, (list, tuple)) else str(hosts)
    port = int(cfg.get("chana.mq.cassandra.pass-through.port", 9042))
    ks = str(cfg.get("chana.mq.cassandra.pass-through.keyspace", "chanamq"))
    user = cfg.get("chana.mq.cassandra.pass-through.user", None)
    password = cfg.get("chana.mq.cassandra.pass-through.password", None)
    if bool(cfg.get("chana.mq.store.cassandra-recover", False)) and not store.queue_ids() and not store.message_ids():
        with CqlClient(host, port, user, password) as cl:
            n = pull(cl, store, keyspace=ks)
        log.info("store filled from Cassandra %s:%d/%s: %s", host, port, ks, n)
    m = CassandraMirror(store, host, port, ks, user, password,
                        interval_s=float(cfg.get("chana.mq.store.cassandra-interval-ms", 50)) / 1000.0).start()
    log.info("store rows written through to Cassandra %s:%d/%s", host, port, ks)
    return m


if __name__ == "__main__":
    sys.exit(main())
