"""Basic.Get pollers for bench/gpu_server_e2e.py --getters, in their own process (the
broker's control plane runs in the bench process: pollers there would compete with it for
the GIL).  Pre-fills one queue per poller, prints "ready", polls Basic.Get (no-ack) until
stdin closes -- ``--pipeline`` Gets in flight per poller, answered inside the steps that
decode them -- then prints one JSON line: [[gets ok, gets empty, seconds], ...]."""
import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from chanamq_amd.client import Connection  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--n", type=int, default=4)
    ap.add_argument("--prefill", type=int, default=200000)
    ap.add_argument("--pipeline", type=int, default=64, help="Basic.Gets in flight per poller")
    a = ap.parse_args()
    c = Connection(port=a.port, vhost="/", timeout=60)
    ch = c.channel()
    for i in range(a.n):
        ch.queue_declare(f"e2e.getq{i}")
        for _ in range(a.prefill // a.n):
            ch.basic_publish("", f"e2e.getq{i}", b"g" * 256)
    c.process(0.5)
    stop = threading.Event()
    out = [None] * a.n

    def poll(i):
        pc = Connection(port=a.port, vhost="/", timeout=60)
        pch = pc.channel()
        ok = empty = 0
        t0 = time.time()
        while not stop.is_set():
            if a.pipeline > 1:
                got, e = pch.basic_get_many(f"e2e.getq{i}", a.pipeline, no_ack=True)
                ok += len(got)
                empty += e
            elif pch.basic_get(f"e2e.getq{i}", no_ack=True) is None:
                empty += 1
            else:
                ok += 1
        out[i] = [ok, empty, time.time() - t0]
        pc.close()

    ths = [threading.Thread(target=poll, args=(i,), daemon=True) for i in range(a.n)]
    for t in ths:
        t.start()
    c.close()
    print("ready", flush=True)
    sys.stdin.read()          # the bench closes our stdin when the load is done
    stop.set()
    for t in ths:
        t.join(30)
    print(json.dumps([o for o in out if o is not None]), flush=True)


if __name__ == "__main__":
    main()
