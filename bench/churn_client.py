"""Control-plane churn next to a data load, for bench/gpu_server_e2e.py --churn, in its own
process (the broker's control plane runs in the bench process).

Two kinds of worker threads run until stdin closes:
  conn  open a connection (handshake + Channel.Open), then Connection.Close -- one cycle
  cons  on a long-lived channel: Basic.Consume (wait for ConsumeOk), Basic.Cancel (wait for
        CancelOk) on a queue of their own that no publisher feeds
  rpc   the RPC client pattern: open a connection, declare a server-named exclusive reply
        queue, bind it, consume it, publish a request routed to it, wait for the reply,
        close (the close deletes the exclusive queue) -- one cycle

Prints "ready" once the queues are declared, then one JSON object at the end: cycles and
seconds per kind, and the latency percentiles (ms) of each cycle.  With the broker's light
control sections none of this drains the step pipeline (server/gpu_broker.py _LightLock)."""
import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from chanamq_amd.client import Connection  # noqa: E402


def pct(xs, p):
    if not xs:
        return None
    xs = sorted(xs)
    return round(xs[min(len(xs) - 1, int(p / 100.0 * len(xs)))] * 1e3, 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--conn-threads", type=int, default=4)
    ap.add_argument("--cons-threads", type=int, default=4)
    ap.add_argument("--rpc-threads", type=int, default=0)
    a = ap.parse_args()
    setup = Connection(port=a.port, vhost="/", timeout=60)
    sch = setup.channel()
    for i in range(a.cons_threads):
        sch.queue_declare(f"churn.q{i}")
    if a.rpc_threads:
        sch.exchange_declare("churn.rpcx", "direct")
    setup.close()
    stop = threading.Event()
    lat = {"conn": [], "cons": [], "cancel": [], "rpc": []}
    cnt = {"conn": 0, "cons": 0, "rpc": 0}
    errs = []
    t_start = [0.0]

    def conn_worker():
        while not stop.is_set():
            t0 = time.perf_counter()
            try:
                c = Connection(port=a.port, vhost="/", timeout=30)
                c.channel()
                c.close()
            except Exception as e:   # counted, the churn goes on
                errs.append(repr(e))
                time.sleep(0.01)
                continue
            lat["conn"].append(time.perf_counter() - t0)
            cnt["conn"] += 1

    def cons_worker(i):
        c = Connection(port=a.port, vhost="/", timeout=30)
        ch = c.channel()
        k = 0
        while not stop.is_set():
            tag = f"churn-{i}-{k}"
            k += 1
            try:
                t0 = time.perf_counter()
                ch.basic_consume(f"churn.q{i}", consumer_tag=tag, no_ack=True)
                t1 = time.perf_counter()
                ch.basic_cancel(tag)
                t2 = time.perf_counter()
            except Exception as e:
                errs.append(repr(e))
                break
            lat["cons"].append(t1 - t0)
            lat["cancel"].append(t2 - t1)
            cnt["cons"] += 1
        try:
            c.close()
        except Exception:
            pass

    def rpc_worker(i):
        k = 0
        while not stop.is_set():
            t0 = time.perf_counter()
            try:
                c = Connection(port=a.port, vhost="/", timeout=30)
                ch = c.channel()
                q = ch.queue_declare("", exclusive=True).queue
                ch.queue_bind(q, "churn.rpcx", q)
                ch.basic_consume(q, consumer_tag="rpc", no_ack=True)
                body = b"req-%d-%d" % (i, k)
                ch.basic_publish("churn.rpcx", q, body)
                got = ch.consume_n(1, timeout=30)
                c.close()
                if got[0].body != body:
                    raise RuntimeError("rpc reply mismatch")
            except Exception as e:
                errs.append(repr(e))
                time.sleep(0.01)
                continue
            k += 1
            lat["rpc"].append(time.perf_counter() - t0)
            cnt["rpc"] += 1

    ths = [threading.Thread(target=conn_worker, daemon=True) for _ in range(a.conn_threads)]
    ths += [threading.Thread(target=rpc_worker, args=(i,), daemon=True) for i in range(a.rpc_threads)]
    ths += [threading.Thread(target=cons_worker, args=(i,), daemon=True) for i in range(a.cons_threads)]
    print("ready", flush=True)
    sys.stdin.readline()       # "go": the load's measured window starts
    t_start[0] = time.perf_counter()
    for t in ths:
        t.start()
    sys.stdin.read()           # the bench closes our stdin when the load is done
    stop.set()
    el = time.perf_counter() - t_start[0]
    for t in ths:
        t.join(30)
    out = dict(seconds=round(el, 3),
               conn_cycles=cnt["conn"], conn_per_s=round(cnt["conn"] / el, 1),
               consume_cancel_cycles=cnt["cons"], consume_cancel_per_s=round(cnt["cons"] / el, 1),
               conn_cycle_ms=dict(p50=pct(lat["conn"], 50), p99=pct(lat["conn"], 99), max=pct(lat["conn"], 100)),
               consume_ok_ms=dict(p50=pct(lat["cons"], 50), p99=pct(lat["cons"], 99), max=pct(lat["cons"], 100)),
               cancel_ok_ms=dict(p50=pct(lat["cancel"], 50), p99=pct(lat["cancel"], 99), max=pct(lat["cancel"], 100)),
               rpc_cycles=cnt["rpc"], rpc_per_s=round(cnt["rpc"] / el, 1),
               rpc_cycle_ms=dict(p50=pct(lat["rpc"], 50), p99=pct(lat["rpc"], 99), max=pct(lat["rpc"], 100)),
               errors=len(errs), error_sample=errs[:3])
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
