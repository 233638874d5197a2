"""One rank of a sharded GPU broker (``python -m chanamq_amd.server.sharded``), started by
``chanamq_amd.parallel.launch`` once per GPU:

    python -m chanamq_amd.parallel.launch 8 -- -m chanamq_amd.server.sharded --port 5672

Each rank owns one MI355X (``--plane gpu``, RCCL between ranks) or a golden CPU plane
(``--plane golden``, gloo; tests).  With ``--reuseport`` all ranks listen on the same port
and the kernel spreads connections over them; otherwise rank r listens on port + r.
Queues are placed on the rank where they are declared; publishes reach them from any
rank through the per-step all-to-all.
"""

import argparse
import json
import os
import signal
import sys
import threading


def main(argv=None):
    ap = argparse.ArgumentParser(prog="chanamq_amd.server.sharded")
    ap.add_argument("--plane", choices=["gpu", "golden"], default="gpu")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=5672)
    ap.add_argument("--reuseport", action="store_true")
    ap.add_argument("--info-dir", default="")
    ap.add_argument("--idle-step-ms", type=float, default=1.0)
    ap.add_argument("--c-max", type=int, default=256)
    ap.add_argument("--store-dir", default="", help="durable store root: rank r keeps <dir>/rank<r>; "
                                                    "survivors adopt a dead rank's durable queues from it")
    ap.add_argument("--no-fsync", action="store_true")
    ap.add_argument("--backend", default="", help="default: nccl (RCCL) for --plane gpu, gloo for golden; "
                                                  "gloo + gpu rehearses several ranks on one GPU")
    args = ap.parse_args(argv)

    from ..parallel.launch import join
    backend = args.backend or ("nccl" if args.plane == "gpu" else "gloo")
    rank, world, store = join(backend)
    if args.plane == "gpu" and backend != "nccl":
        import torch
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", rank)) % max(1, torch.cuda.device_count()))
    from ..parallel.comm import Comm
    from ..parallel.node import ShardedNode
    if args.plane == "gpu":
        import torch
        from ..engine.dataplane import GpuDataPlane
        plane = GpuDataPlane(device=torch.cuda.current_device(), world=world, rank=rank, worker=rank,
                             c_max=args.c_max, chpc=8, q_max=1024, cons_max=4096, seg_max=args.c_max,
                             cmd_max=1 << 16, deliv_max=1 << 16, msg_max=1 << 20, ingress_cap=32 << 20,
                             egress_cap=64 << 20, log_bytes=2 << 30, ring_pool=1 << 24, tb_max=1024,
                             default_queue_capacity=1 << 14, persist=1)   # persist: store rows and remote-consumer acks
    else:
        from ..engine.golden import GoldenDataPlane
        plane = GoldenDataPlane(world=world, rank=rank, c_max=args.c_max, chpc=8, q_max=1024,
                                default_queue_capacity=1 << 14, ring_pool=1 << 24, persist=bool(args.store_dir))
    node = ShardedNode(plane, Comm(store=store, backend=backend, timeout_s=60, wait_s=20))
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
    broker = GpuBroker(plane, host=args.host, port=port, idle_step_ms=args.idle_step_ms, node=node,
                       reuseport=args.reuseport, ingress_bytes=32 << 20, store=st).start()
    node.persistence = broker.persistence if st is not None else None
    if args.info_dir:
        # written then renamed: a watcher polling for the file never reads it half-written
        path = os.path.join(args.info_dir, f"rank{rank}.json")
        with open(path + ".tmp", "w") as f:
            json.dump({"rank": rank, "world": world, "port": broker.port}, f)
        os.replace(path + ".tmp", path)
    stop = threading.Event()
    for sig in (signal.SIGINT, signal.SIGTERM):
        signal.signal(sig, lambda *a: stop.set())
    stop.wait()
    broker.stop()
    node.close()
    if st is not None:
        st.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
