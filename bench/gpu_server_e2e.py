#!/usr/bin/env python3
"""End-to-end over TCP: the native load generator (csrc/core/loadgen.cpp) against the
GPU-data-path server (server/gpu_broker.py + GpuDataPlane) on one MI355X.  Unlike
bench.py (which feeds pre-rendered wire bytes straight into the data plane), this includes
the Python socket front end, so it measures the full broker as a client sees it.

python bench/gpu_server_e2e.py [--seconds S] [--out FILE]
"""

import argparse
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from chanamq_amd.broker import load  # noqa: E402

SPECS = {
    "topic_16q_1KB_auto_ack": dict(producers=4, consumers=16, queues=16, msg_size=1024, auto_ack=True,
                                   prefetch=5000, exchange_type="topic"),
    "direct_1p1c_256B": dict(producers=1, consumers=1, msg_size=256, auto_ack=True, prefetch=5000),
    "direct_4p4c_1KB_manual_ack": dict(producers=4, consumers=4, msg_size=1024, auto_ack=False, prefetch=1000),
    # BASELINE config 4 shape: durable queue, delivery-mode 2, 4 KB, publisher confirms, manual ack
    "config4_durable_4KB_confirms": dict(producers=1, consumers=1, msg_size=4096, auto_ack=False, prefetch=1000,
                                         persistent=True, durable=True, confirm=True),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--out", default="")
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    import torch
    from chanamq_amd.engine.dataplane import GpuDataPlane
    from chanamq_amd.server.gpu_broker import GpuBroker
    assert torch.cuda.is_available()
    core = load()
    results = {}
    for name, spec in SPECS.items():
        if args.only and args.only not in name:
            continue
        persist = bool(spec.get("persistent"))
        plane = GpuDataPlane(c_max=256, chpc=8, q_max=256, cons_max=1024, seg_max=256, cmd_max=1 << 16,
                             deliv_max=1 << 16, msg_max=1 << 20, ucap=8192, deliver_cap=8192,
                             ingress_cap=64 << 20, egress_cap=128 << 20, log_bytes=4 << 30, ring_pool=1 << 24,
                             tb_max=256, default_queue_capacity=1 << 18, persist=int(persist),
                             persist_max=1 << 15, persist_bytes=256 << 20)
        store = None
        if persist:
            store = core.Store()
            store.open(tempfile.mkdtemp(prefix="cmq-gpu-store-"), True)
        b = GpuBroker(plane, idle_step_ms=0.5, store=store).start()
        try:
            r = core.run_load(dict(port=b.port, seconds=args.seconds, queue=f"e2e.{name}", exchange=f"e2e.x.{name}",
                                   **spec))
        finally:
            b.stop()
            if store is not None:
                store.close()
        lc = getattr(plane, "last_counters", {}) or {}
        r.update(name=name, spec=spec, recv_msgs_per_s=r["received"] / r["elapsed"],
                 sent_msgs_per_s=r["sent"] / r["elapsed"], steps=b.stats["steps"], server=dict(b.stats),
                 last_step={k: lc.get(k) for k in ("n_pubs", "n_deliv", "n_ring_full", "n_live_msgs", "live_bytes",
                                                   "n_dropped_nomem", "egress_bytes")})
        results[name] = r
        print(json.dumps({k: r[k] for k in ("name", "recv_msgs_per_s", "sent_msgs_per_s", "p50_us", "p99_us",
                                            "steps", "error", "server", "last_step")}), flush=True)
        del plane
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"meta": {"transport": "loopback TCP", "front_end": "python selectors (1 thread)",
                                "data_plane": "HIP gfx950"}, "results": results}, f, indent=1)


if __name__ == "__main__":
    main()
