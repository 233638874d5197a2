"""Timed cold paging with live traffic.

One GPU server with small body tiers (HBM log ``--log-mb``, pinned host spill ring
``--ring-mb``) and the cold store on disk.  Phase 1 publishes a backlog several times the
two in-memory tiers to one queue (paced so nothing is nacked: the tiers move bodies while
the publishers run).  Phase 2 drains it with ``--drainers`` consumers while a paced 1P1C
stream of 1 KB messages runs on another queue; the cold-in rate is what the cold thread
paged back from disk during the drain, the live stream's publish->deliver latency is the
native load generator's.

Both tiers ride the steps (k_dequeue's in-step spill, the cold thread's engine side
operations), so the stepper pause count must not move during the run.  Before the drain a
``--hold-s`` phase runs the same live stream next to the resting backlog.  Bodies of a
sample of the drained messages are checked against the load generator's fill pattern.
Reference: MessageEntity.scala:82-102,174-186 (bodies leave memory, come back on demand).

    python bench/cold_paging.py --backlog-s 4 --drain-s 12 --out gpurun_out/cold.json
"""

import argparse
import json
import os
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from chanamq_amd.broker import load  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-mb", type=int, default=256)
    ap.add_argument("--ring-mb", type=int, default=512)
    ap.add_argument("--body", type=int, default=16 << 10)
    ap.add_argument("--producers", type=int, default=4)
    ap.add_argument("--rate", type=float, default=8000.0, help="backlog msgs/s per producer")
    ap.add_argument("--backlog-s", type=float, default=4.0)
    ap.add_argument("--drain-s", type=float, default=12.0, help="live stream duration (the drain runs under it)")
    ap.add_argument("--drainers", type=int, default=4)
    ap.add_argument("--live-rate", type=float, default=10000.0, help="live msgs/s (1 KB, 1P1C)")
    ap.add_argument("--io-threads", type=int, default=4)
    ap.add_argument("--deliver-cap-bytes", type=int, default=1 << 20,
                    help="per-consumer egress per step (the server's chana.mq.gpu.deliver-cap-bytes; 0 = off)")
    ap.add_argument("--cold-sync", action="store_true", help="cold tier between paused steps (the old path)")
    ap.add_argument("--hold-s", type=float, default=6.0, help="live stream next to the resting backlog first")
    ap.add_argument("--out", default="")
    args = ap.parse_args()

    import torch  # noqa: F401  (HIP runtime up before the plane)
    from chanamq_amd.client import Connection
    from chanamq_amd.engine.dataplane import GpuDataPlane
    from chanamq_amd.server.gpu_broker import GpuBroker
    core = load()
    cold_dir = tempfile.mkdtemp(prefix="cmq-cold-", dir=os.environ.get("TMPDIR", "/tmp"))
    plane = GpuDataPlane(c_max=64, chpc=8, q_max=64, cons_max=256, seg_max=64, cmd_max=1 << 16, deliv_max=1 << 16,
                         msg_max=1 << 20, ucap=4096, deliver_cap=4096, ingress_cap=32 << 20, egress_cap=64 << 20,
                         log_bytes=args.log_mb << 20, log_block=1 << 20, spill_bytes=args.ring_mb << 20,
                         ring_pool=1 << 23, default_queue_capacity=1 << 20, carry_cap=1 << 20,
                         deliver_cap_bytes=args.deliver_cap_bytes)
    b = GpuBroker(plane, idle_step_ms=0.5, io="pipeline", io_threads=args.io_threads, mem_high_watermark=0,
                  cold_dir=cold_dir, cold_hot=4096, cold_window=4096, cold_beside=not args.cold_sync).start()
    out = dict(config=vars(args), cold_dir=cold_dir)
    try:
        # ---- phase 1: the backlog
        t0 = time.time()
        # (default exchange: each phase's load generator routes by queue name only)
        r1 = core.run_load(dict(port=b.port, seconds=args.backlog_s, warmup=0.0, queue="cold.deep", exchange="",
                                producers=args.producers, consumers=0, msg_size=args.body, rate=args.rate,
                                threads=args.producers))
        pub = int(r1["sent"])
        deadline, last, since = time.time() + 20, -1, time.time()   # the steps caught up
        while time.time() < deadline and time.time() - since < 1.0:
            b._sync_fe_stats()
            cur = b._fe_stats.get("published", 0)
            if cur >= pub:
                break
            if cur != last:
                last, since = cur, time.time()
            time.sleep(0.05)
        # (the load generator counts the last batch of each producer as sent even when its
        # connection closed mid-batch: the backlog is what the broker published)
        out["fe_published"] = b._fe_stats.get("published", 0)
        pub = min(pub, int(out["fe_published"]))
        time.sleep(0.5)   # the cold thread's last moves
        st1 = dict(b.stats)
        out["backlog"] = dict(published=pub, seconds=round(time.time() - t0, 2), bytes=pub * args.body,
                              cold_out_bytes=st1.get("cold_out_bytes", 0), spilled_bytes=st1.get("spilled_bytes", 0),
                              on_disk=b.cold.bytes_on_disk(), nacked=int(r1.get("nacked", 0)), error=r1["error"])
        print("backlog", json.dumps(out["backlog"]), flush=True)
        # ---- the live stream next to the resting backlog (tiers full, nothing drained)
        if args.hold_s > 0:
            st_h = dict(b.stats)
            h = core.run_load(dict(port=b.port, seconds=args.hold_s, warmup=1.0, queue="cold.hold", exchange="",
                                   producers=1, consumers=1, msg_size=1024, rate=args.live_rate, threads=2,
                                   prefetch=1000))
            out["hold"] = {k: h.get(k) for k in ("sent", "received", "elapsed", "p50_us", "p95_us", "p99_us", "error")}
            out["hold"]["pauses"] = b.stats.get("pauses", 0) - st_h.get("pauses", 0)
            print("hold", json.dumps(out["hold"]), flush=True)
        # ---- phase 2: drain under live traffic
        got = [0] * args.drainers
        bad = [0]
        bad_ex = []
        checked = [0]
        stop = [False]

        def drain(k):
            # (every drainer stays until the whole backlog arrived: one that left early would
            # drop the no-ack deliveries still on its way)
            c = Connection(port=b.port)
            ch = c.channel()
            ch.basic_qos(prefetch_count=256)
            ch.basic_consume("cold.deep", f"drain{k}", no_ack=True)
            try:
                while sum(got) < pub and not stop[0]:
                    c.process(0.02)
                    ds = list(ch.deliveries)
                    ch.deliveries.clear()
                    for i, d in enumerate(ds):
                        if (got[k] + i) % 97 == 0:   # sample: the load generator's 'x' fill after its stamp
                            body = d.body
                            checked[0] += 1
                            if len(body) != args.body or body[8:] != fill:
                                bad[0] += 1
                                if len(bad_ex) < 12:
                                    import numpy as np
                                    a = np.frombuffer(body, np.uint8)
                                    w = np.nonzero(a[8:] != ord("x"))[0] + 8 if len(a) > 8 else np.array([0])
                                    bad_ex.append(dict(len=len(body), first=int(w[0]) if len(w) else -1,
                                                       last=int(w[-1]) if len(w) else -1, n=int(len(w)),
                                                       at=body[int(w[0]):int(w[0]) + 24].hex() if len(w) else "",
                                                       redelivered=bool(getattr(d.method, "redelivered", False)),
                                                       tag=getattr(d.method, "consumer_tag", None),
                                                       rk=getattr(d.method, "routing_key", None),
                                                       dtag=getattr(d.method, "delivery_tag", None),
                                                       drainer=k, nth=got[k] + i))
                    got[k] += len(ds)
            finally:
                c.close()

        fill = b"x" * (args.body - 8)
        live = {}

        def live_run():
            live.update(core.run_load(dict(port=b.port, seconds=args.drain_s, warmup=1.0, queue="cold.live", exchange="",
                                           producers=1, consumers=1, msg_size=1024, rate=args.live_rate,
                                           threads=2, prefetch=1000)))
        lt = threading.Thread(target=live_run)
        lt.start()
        time.sleep(1.0)   # the live stream's topology and warm-up
        st_a = dict(b.stats)
        b._sync_fe_stats()
        fe_a = dict(b._fe_stats)
        td = time.time()
        ths = [threading.Thread(target=drain, args=(k,)) for k in range(args.drainers)]
        for t in ths:
            t.start()
        while sum(got) < pub and time.time() - td < args.drain_s + 120:
            time.sleep(0.01)
        drain_s = time.time() - td
        stop[0] = True
        for t in ths:
            t.join(timeout=10)
        st_b = dict(b.stats)
        b._sync_fe_stats()
        fe_b = dict(b._fe_stats)
        lt.join()
        stop[0] = True
        n = sum(got)
        cin = st_b.get("cold_in_bytes", 0) - st_a.get("cold_in_bytes", 0)
        out["drain"] = dict(received=n, of=pub, seconds=round(drain_s, 2), msgs_per_s=round(n / drain_s),
                            body_mb_per_s=round(n * args.body / drain_s / 2**20, 1),
                            cold_in_bytes=cin, cold_in_mb_per_s=round(cin / drain_s / 2**20, 1),
                            bodies_checked=checked[0], bodies_bad=bad[0], bad_examples=bad_ex,
                            pauses=st_b.get("pauses", 0) - st_a.get("pauses", 0),
                            cold_side_ops=st_b.get("cold_side_ops", 0) - st_a.get("cold_side_ops", 0),
                            cold_errors=st_b.get("cold_errors", 0),
                            # the front end during the drain: step period / IO phase / result wait
                            # (log2 us bins) and the IO threads' busiest phase
                            front_end={k: [x - y for x, y in zip(fe_b[k], fe_a[k])] for k in
                                       ("h_period_us_log2", "h_io_us_log2", "h_wait_us_log2", "h_submit_us_log2")
                                       if k in fe_b and k in fe_a})
        out["live"] = {k: live.get(k) for k in ("sent", "received", "elapsed", "p50_us", "p95_us", "p99_us", "error")}
        print("drain", json.dumps(out["drain"]), flush=True)
        print("live", json.dumps(out["live"]), flush=True)
    finally:
        b.stop()
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
