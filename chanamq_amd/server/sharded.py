"""One rank of a sharded GPU broker (``python -m chanamq_amd.server.sharded``), started by
``chanamq_amd.parallel.launch`` once per GPU:

    python -m chanamq_amd.parallel.launch 8 -- -m chanamq_amd.server.sharded --port 5672

Each rank owns one MI355X (``--plane gpu``) or a golden CPU plane (``--plane golden``,
gloo; tests).  With ``--reuseport`` all ranks listen on the same port and the kernel
spreads connections over them; otherwise rank r listens on port + r.  Queues are placed
on the rank where they are declared; publishes reach them from any rank through the
per-step exchange, consumers on any rank reach any queue through device links.

``--io pipeline`` (GPU default): the native front end (csrc/core/frontend.cpp) steps the
rank in lockstep with its peers, the engine moves each step's cross-rank records itself
(``--backend nccl``: RCCL send/recv over xGMI; ``--backend gloo``: host shared memory,
several ranks on one GPU), replicated control ops are synced at flagged steps on a host
(gloo) control group, and a peer that stops answering is failed over.  ``--io native``:
the round-1 Python lockstep loop (golden planes always use it).
"""

import argparse
import json
import os
import signal
import sys
import threading
import uuid


def sharded_plane_config(cfg, args, world, rank, pipeline):
    """(GpuDataPlane kwargs, GpuBroker kwargs) of one rank from ``chana.mq.gpu.*`` -- the
    same keys and defaults as the single-GPU launcher (AMQPServer.scala:52-70: every node
    boots from the same HOCON) -- plus the rank's place in the group.  Command-line flags
    override their keys.  Every rank keeps store rows (persist) for failover adoption."""
    plane, broker = cfg.gpu_config(single=False)
    plane.pop("device", None)   # each rank drives its own LOCAL_RANK GPU
    if args.c_max:
        plane["c_max"] = args.c_max
    plane["seg_max"] = min(plane["seg_max"], plane["c_max"])
    plane.update(world=world, rank=rank, worker=rank, persist=1, native_xchg=int(pipeline), links=int(pipeline))
    broker.pop("io", None)      # --io decides the front end of a sharded rank
    if args.idle_step_ms is not None:
        broker["idle_step_ms"] = args.idle_step_ms
    if args.io_threads is not None:
        broker["io_threads"] = args.io_threads
    return plane, broker


def main(argv=None):
    ap = argparse.ArgumentParser(prog="chanamq_amd.server.sharded")
    ap.add_argument("--config", action="append", default=[],
                    help="HOCON file over conf/reference.conf (every rank reads the same files)")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE")
    ap.add_argument("--plane", choices=["gpu", "golden"], default="gpu")
    ap.add_argument("--io", choices=["pipeline", "native"], default="pipeline",
                    help="gpu plane: pipeline = native front end + native exchange; native = Python lockstep loop")
    ap.add_argument("--host", default=None, help="default chana.mq.amqp.server.interface")
    ap.add_argument("--port", type=int, default=None, help="default chana.mq.amqp.server.port")
    ap.add_argument("--reuseport", action="store_true")
    ap.add_argument("--info-dir", default="")
    ap.add_argument("--idle-step-ms", type=float, default=None, help="default chana.mq.gpu.idle-step-ms")
    ap.add_argument("--io-threads", type=int, default=None, help="default chana.mq.gpu.io-threads")
    ap.add_argument("--c-max", type=int, default=None, help="default chana.mq.gpu.max-connections")
    ap.add_argument("--store-dir", default=None, help="durable store root (default chana.mq.store.dir): rank r "
                                                      "keeps <dir>/rank<r>; survivors adopt a dead rank's durable "
                                                      "queues from it")
    ap.add_argument("--no-fsync", action="store_true")
    ap.add_argument("--backend", default="", help="default: nccl (RCCL) for --plane gpu, gloo for golden; "
                                                  "gloo + gpu rehearses several ranks on one GPU")
    ap.add_argument("--xchg", choices=["auto", "rccl", "shm"], default="auto",
                    help="pipeline: the engine's exchange backend (auto: rccl with --backend nccl, else shm); rccl "
                         "under gloo runs the RCCL code path through CHANAMQ_RCCL_LIB (the tests' stand-in)")
    ap.add_argument("--async-x", type=int, default=0,
                    help="1: each step's exchange on the engine's exchange thread (phase B waits on the device)")
    ap.add_argument("--xchg-timeout-ms", type=int, default=15000,
                    help="pipeline: a peer silent this long in an exchange is failed over")
    ap.add_argument("--hb-timeout-s", type=float, default=3.0)
    ap.add_argument("--tls-port", type=int, default=-1, help="AMQPS on tls-port + rank (0: ephemeral; -1: off)")
    ap.add_argument("--tls-cert", default="")
    ap.add_argument("--tls-key", default="")
    args = ap.parse_args(argv)
    from ..utils.config import Config
    cfg = Config.load(args.config, dict(kv.split("=", 1) for kv in args.set))
    bc = cfg.broker_config()
    if args.host is None:
        args.host = bc["host"]
    if args.port is None:
        args.port = bc["port"]
    if args.store_dir is None:
        args.store_dir = bc["data_dir"]
    if args.no_fsync is False and not bc["fsync"]:
        args.no_fsync = True

    from ..parallel.launch import ENV_STORE, join
    backend = args.backend or ("nccl" if args.plane == "gpu" else "gloo")
    pipeline = args.plane == "gpu" and args.io == "pipeline"
    # pipelined ranks never run collectives on the default group: it is gloo (control
    # only) whatever the data backend
    rank, world, store = join("gloo" if pipeline else backend)
    if args.plane == "gpu" and (backend != "nccl" or pipeline):
        import torch
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", rank)) % max(1, torch.cuda.device_count()))
    from ..parallel.comm import Comm
    from ..parallel.membership import Membership
    from ..parallel.node import ShardedNode
    gpu_kw, broker_kw = sharded_plane_config(cfg, args, world, rank, pipeline)
    if args.plane == "gpu":
        import torch
        from ..engine.dataplane import GpuDataPlane
        plane = GpuDataPlane(device=torch.cuda.current_device(), **gpu_kw)
    else:   # the CPU model (tests): small tables whatever the GPU sizing says
        from ..engine.golden import GoldenDataPlane
        plane = GoldenDataPlane(persist=bool(args.store_dir), world=world, rank=rank,
                                c_max=args.c_max or 256, chpc=8, q_max=1024, default_queue_capacity=1 << 14,
                                ring_pool=1 << 24)
    comm = Comm(store=store, backend="gloo" if pipeline else backend, timeout_s=60, wait_s=20)
    node = ShardedNode(plane, comm, membership=Membership(store, rank, world, timeout_s=args.hb_timeout_s))
    if pipeline:
        xkind = args.xchg if args.xchg != "auto" else ("rccl" if backend == "nccl" else "shm")
        shm_base = "cmq-x-" + os.environ.get(ENV_STORE, "local").replace(":", "-").replace(".", "-")

        def rebuild_xchg(live, epoch):
            """The engine's exchange over the live ranks (startup: epoch 0; after a failover
            the survivors build a new RCCL communicator / shared segment)."""
            if xkind == "rccl":
                key = f"xchg/{epoch}/uid"
                if rank == min(live):
                    store.set(key, plane.xchg_unique_id())
                uid = store.get(key)
                plane.xchg_setup("rccl", uid, live, args.xchg_timeout_ms, failover=True, async_x=bool(args.async_x))
            else:
                # a fresh segment name per launch and epoch, chosen by the lowest live rank: a
                # segment left by a killed earlier run (same store address) is never reused
                key = f"xchg/{epoch}/shm"
                if rank == min(live):
                    store.set(key, f"{shm_base}-{os.getpid()}-{uuid.uuid4().hex[:12]}-e{epoch}")
                name = store.get(key).decode()
                plane.xchg_setup("shm", name, live, args.xchg_timeout_ms, failover=True, async_x=bool(args.async_x))
        rebuild_xchg(list(range(world)), 0)
        node.rebuild_xchg = rebuild_xchg
    st = None
    if args.store_dir:
        from ..store import open_store as _open, rank_dir

        def open_store(r):
            return _open(rank_dir(args.store_dir, r), not args.no_fsync)
        st = open_store(rank)
        node.peer_store = open_store
    from .gpu_broker import GpuBroker
    # --port 0: every rank takes an ephemeral port (reported through --info-dir)
    port = args.port if (args.reuseport or args.port == 0) else args.port + rank
    broker = GpuBroker(plane, host=args.host, port=port, node=node, reuseport=args.reuseport,
                       ingress_bytes=min(32 << 20, plane.info["ingress_cap"]) if args.plane == "gpu" else 32 << 20,
                       store=st, io="pipeline" if pipeline else "native", heartbeat=bc["heartbeat"],
                       frame_max=bc["frame_max"], channel_max=bc["channel_max"] or 2047, **broker_kw).start()
    node.persistence = broker.persistence if st is not None else None
    tls = None
    if args.tls_port >= 0:   # AMQPS per rank: the TLS terminator in front of this rank's front end
        from ..broker import load
        tls = load().TlsProxy(dict(host=args.host, port=args.tls_port + rank if args.tls_port else 0,
                                   upstream_port=broker.port, cert=args.tls_cert, key=args.tls_key, p12="",
                                   p12_password=""))
        tls.start()
    def write_info():
        if not args.info_dir:
            return
        # written then renamed: a watcher polling for the file never reads it half-written
        path = os.path.join(args.info_dir, f"rank{rank}.json")
        fes = getattr(broker, "_fe_stats", None) or {}
        with open(path + ".tmp", "w") as f:
            json.dump({"rank": rank, "world": world, "port": broker.port,
                       "tls_port": tls.port if tls is not None else None, "io": broker.io,
                       "stats": dict(broker.stats), "failovers": len(node.failovers),
                       "plane": {k: plane.info[k] for k in ("log_bytes", "msg_max", "c_max", "q_max", "ingress_cap",
                                                            "egress_cap", "spill_bytes")
                                 if hasattr(plane, "info") and k in plane.info},
                       "front_end": {k: v for k, v in fes.items() if k != "lat_hist"},
                       # (diagnostics) control ops not yet synced, deferred replies, and with
                       # CHANAMQ_CTL_TRACE=1 the tail of the control trace
                       "control": {"outbox": len(node.log.outbox), "applied": node.log.applied,
                                   "deferred": len(getattr(broker, "_deferred", {}) or {}),
                                   "trace": [repr(t) for t in list(broker.ctl_trace or [])[-40:]]}}, f)
        os.replace(path + ".tmp", path)
    write_info()
    stop = threading.Event()
    for sig in (signal.SIGINT, signal.SIGTERM):
        signal.signal(sig, lambda *a: stop.set())
    rc = 0
    while not stop.wait(0.5):
        write_info()
        if not broker._running:   # the engine failed: leave, the peers fail this rank over
            rc = 3
            break
    if tls is not None:
        tls.stop()
    broker.stop()
    node.close()
    if st is not None:
        st.close()
    if rc:
        os._exit(rc)
    return 0


if __name__ == "__main__":
    sys.exit(main())
