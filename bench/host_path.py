#!/usr/bin/env python3
"""Host-path benchmarks (no GPU): BASELINE.json config 1 and the reference's PerfTest specs
(chana-mq-test/perf/publish-consume-spec*.js), driven by the native load generator against
the native broker over loopback TCP.

python bench/host_path.py [--seconds S] [--out FILE]
"""

import argparse
import json
import os
import platform
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from chanamq_amd.broker import load  # noqa: E402

SPECS = {
    # BASELINE config 1: 1 direct exchange, 1 queue, 1P/1C, 256 B, non-persistent (auto-ack)
    "config1_direct_1p1c_256B": dict(producers=1, consumers=1, msg_size=256, auto_ack=True, prefetch=5000),
    # same, rate-limited below saturation so latency is not dominated by queue build-up
    "config1_direct_1p1c_256B_paced": dict(producers=1, consumers=1, msg_size=256, auto_ack=True, prefetch=5000,
                                           rate=200000),
    # publish-consume-spec.js: 3P/3C, minMsgSize 0, manual ack, prefetch 5000
    "perftest_3p3c_manual_ack": dict(producers=3, consumers=3, msg_size=0, auto_ack=False, prefetch=5000),
    # publish-consume-spec-a.js: auto-ack
    "perftest_3p3c_auto_ack": dict(producers=3, consumers=3, msg_size=0, auto_ack=True, prefetch=5000),
    # publish-consume-spec-p.js / -a-p.js: 3P/1C persistent (durable queue)
    "perftest_3p1c_persistent_manual": dict(producers=3, consumers=1, msg_size=0, auto_ack=False, prefetch=5000,
                                            persistent=True, durable=True),
    "perftest_3p1c_persistent_auto": dict(producers=3, consumers=1, msg_size=0, auto_ack=True, prefetch=5000,
                                          persistent=True, durable=True),
    # BASELINE config 4 shape on the host path: durable, 4 KB persistent, publisher confirms
    "config4_durable_4KB_confirms": dict(producers=1, consumers=1, msg_size=4096, auto_ack=False, prefetch=1000,
                                         persistent=True, durable=True, confirm=True),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--only", default="")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    core = load()
    results = {}
    for name, spec in SPECS.items():
        if args.only and args.only not in name:
            continue
        d = tempfile.mkdtemp(prefix="cmq-bench-")
        b = core.Broker({"port": 0, "host": "127.0.0.1", "heartbeat": 0, "data_dir": d, "fsync": True})
        b.start()
        try:
            r = core.run_load(dict(port=b.port, seconds=args.seconds, queue=f"bq.{name}", exchange=f"bx.{name}",
                                   **spec))
        finally:
            b.stop()
        r.update(name=name, spec=spec, recv_msgs_per_s=r["received"] / r["elapsed"],
                 sent_msgs_per_s=r["sent"] / r["elapsed"])
        results[name] = r
        print(json.dumps({k: r[k] for k in ("name", "recv_msgs_per_s", "sent_msgs_per_s", "p50_us", "p99_us",
                                            "error")}))
    meta = {"hardware": platform.processor() or platform.machine(), "cpus": os.cpu_count(),
            "transport": "loopback TCP", "broker": "chanamq_amd native (1 event-loop thread)",
            "seconds": args.seconds}
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"meta": meta, "results": results}, f, indent=1)


if __name__ == "__main__":
    main()
