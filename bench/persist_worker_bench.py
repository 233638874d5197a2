"""Config-4 persistence path on the CPU: the native PersistWorker (csrc/core/persist.cpp)
applies the device's per-step persist / consumed records to the store (WAL + group
commit).  Synthetic steps shaped like BASELINE config 4 (4 KB persistent messages,
durable queues, manual ack two steps after delivery); reports rows/s the worker sustains.

    python bench/persist_worker_bench.py [--msgs-per-step 512] [--steps 400] [--fsync]
"""
import argparse
import json
import os
import struct
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from chanamq_amd.broker import load  # noqa: E402
from chanamq_amd.engine.layout import CONSUMED_REC  # noqa: E402


def persist_records(mids, q_of, qpos, body):
    out = bytearray()
    ex, rk, props = b"e2e.x", b"k", b"\x10\x00\x02"
    for mid, q, pos in zip(mids, q_of, qpos):
        payload = ex + rk + props + body
        size = 48 + ((len(payload) + 7) & ~7)
        out += struct.pack("<qqQqIIHBBI", mid, 0, pos, 0, q, len(body), len(props), len(ex), len(rk), size)
        out += payload + b"\0" * (size - 48 - len(payload))
    return bytes(out)


def consumed_records(mids, q_of, qpos, kind):
    a = np.zeros(len(mids), CONSUMED_REC)
    for i, (m, q, p) in enumerate(zip(mids, q_of, qpos)):
        a[i] = (m, p, q, kind, (0, 0))
    return a.tobytes()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--msgs-per-step", type=int, default=512)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--queues", type=int, default=4)
    ap.add_argument("--body", type=int, default=4096)
    ap.add_argument("--fsync", action="store_true")
    ap.add_argument("--dir", default="")
    ap.add_argument("--window", type=int, default=1,
                    help="steps in flight before the producer waits for commits (1 = commit every step "
                         "before the next; the pipelined front end keeps stepping while a commit runs)")
    ap.add_argument("--group-ms", type=float, default=0.0, help="PersistWorker.set_group_delay")
    a = ap.parse_args()
    core = load()
    d = a.dir or tempfile.mkdtemp()
    st = core.Store()
    st.open(os.path.join(d, "store"), a.fsync)
    w = core.PersistWorker(st)
    if a.group_ms:
        w.set_group_delay(a.group_ms)
    for q in range(a.queues):
        w.set_queue(q, f"AMQ.DEFAULT-_.cfg4.q{q}")
    w.start()
    body = os.urandom(a.body)
    n = a.msgs_per_step
    hist = []          # per step: (mids, qs, pos)
    pos = [0] * a.queues
    nxt = 1
    batches = []
    for s in range(a.steps + 2):
        batch_p, batch_c = b"", b""
        if s < a.steps:
            mids = list(range(nxt, nxt + n))
            nxt += n
            qs = [m % a.queues for m in mids]
            ps = []
            for q in qs:
                ps.append(pos[q])
                pos[q] += 1
            hist.append((mids, qs, ps))
            batch_p = persist_records(mids, qs, ps, body)
        if s >= 1 and s - 1 < len(hist):      # delivered to manual-ack consumers one step later
            batch_c += consumed_records(*hist[s - 1], 3)
        if s >= 2 and s - 2 < len(hist):      # acked the step after
            batch_c += consumed_records(*hist[s - 2], 0)
        batches.append((batch_p, batch_c))
    t0 = time.perf_counter()                   # the records are prebuilt: only the worker is timed
    for s, (batch_p, batch_c) in enumerate(batches):
        w.submit(s + 1, batch_p, batch_c)
        if (s + 1) % a.window == 0:
            w.drain()                          # confirm gating: held egress waits for the commit
    w.drain()
    dt = time.perf_counter() - t0
    stats = w.stats()
    w.stop()
    st.close()
    msgs = a.steps * n
    print(json.dumps({"msgs": msgs, "seconds": round(dt, 3), "msgs_per_s": round(msgs / dt),
                      "body_MBps": round(msgs * a.body / dt / 1e6, 1), "fsync": a.fsync, "window": a.window, **stats}))


if __name__ == "__main__":
    main()
