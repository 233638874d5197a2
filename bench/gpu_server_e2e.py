#!/usr/bin/env python3
"""End-to-end over TCP: the native load generator (csrc/core/loadgen.cpp, epoll threads)
against the GPU-data-path server (server/gpu_broker.py + GpuDataPlane) on one MI355X.
Unlike bench.py (pre-rendered wire bytes handed straight to the data plane), this is the
broker as a client sees it: loopback TCP, the front end, the control plane, the GPU.

Front ends: ``pipeline`` (native IO threads + stepper, csrc/core/frontend.cpp; swept over
--io-threads) and ``native`` (round-1 Python step loop over the C++ gateway) for reference.
Latency = publish->deliver measured by the consumers from the send timestamp carried in
every message body; ``--paced`` re-runs a spec at a fraction of its measured throughput.

python bench/gpu_server_e2e.py [--seconds S] [--only NAME] [--io-threads 1,2,4,8] [--out FILE]
"""

import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from chanamq_amd.broker import load  # noqa: E402

SMALL_CONF = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "sharded_small.conf")

SPECS = {
    # BASELINE config 2 over TCP: 1 topic exchange, 16 bound queues, 1 KB, auto-ack
    "config2_topic_16q_1KB_auto_ack": dict(producers=16, consumers=16, queues=16, msg_size=1024, auto_ack=True,
                                           prefetch=5000, exchange_type="topic"),
    # BASELINE config 1 shape through the GPU server (the round-1 1P1C starvation case)
    "direct_1p1c_256B": dict(producers=1, consumers=1, msg_size=256, auto_ack=True, prefetch=5000),
    "direct_4p4c_1KB_manual_ack": dict(producers=4, consumers=4, queues=4, msg_size=1024, auto_ack=False,
                                       prefetch=1000),
    # BASELINE config 4: durable queues, delivery-mode 2, 4 KB, publisher confirms, manual ack
    "config4_durable_4KB_confirms": dict(producers=16, consumers=4, queues=4, msg_size=4096, auto_ack=False,
                                         prefetch=1000, persistent=True, durable=True, confirm=True,
                                         confirm_window=512),
    # BASELINE config 5 on one GPU: 64P x 64C manual ack, every 2nd ack of each consumer is
    # Basic.Nack(multiple, requeue) (redelivery storm); a 256 MB memory watermark turns
    # producers off with Channel.Flow and back on below 128 MB
    "config5_storm_64p64c_nack_flow": dict(producers=64, consumers=64, queues=16, msg_size=1024, auto_ack=False,
                                           prefetch=512, nack_every=2,
                                           _broker=dict(mem_high_watermark=256 << 20)),
}


def plane_for(spec):
    from chanamq_amd.engine.dataplane import GpuDataPlane
    persist = bool(spec.get("persistent"))
    return GpuDataPlane(c_max=512, chpc=8, q_max=256, cons_max=1024, seg_max=512, cmd_max=1 << 17,
                        deliv_max=1 << 17, msg_max=1 << 21, ucap=8192, deliver_cap=8192,
                        ingress_cap=64 << 20, egress_cap=160 << 20, log_bytes=8 << 30, ring_pool=1 << 27,
                        spill_bytes=SIZING.get("spill_bytes", 8 << 30),   # (default tiering: old bodies leave HBM)
                        tb_max=256, default_queue_capacity=1 << 20, persist=int(persist),
                        persist_max=1 << 16, persist_bytes=512 << 20, carry_cap=SIZING["carry_cap"],
                        **SIZING.get("plane_cfg", {}))


def thread_cpu():
    """CPU seconds (user + system) of this process's threads, grouped by name prefix
    (cmq-io / cmq-stepper = front end, lg-c / lg-p = load generator consumers / producers)."""
    out = {}
    tck = os.sysconf("SC_CLK_TCK")
    for tid in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{tid}/stat") as f:
                st = f.read()
        except OSError:
            continue
        name = st[st.index("(") + 1:st.rindex(")")]
        f = st[st.rindex(")") + 2:].split()
        key = name.rstrip("0123456789")
        out[key] = out.get(key, 0.0) + (int(f[11]) + int(f[12])) / tck
    return out


FE_CFG = {}
BROKER_CFG = {}
# per-connection bytes per step (the front end reads at most this, and at most the room
# left in the connection's device carry, so two steps in flight need carry >= 2x): the
# batch a step can take from one producer, so the ceiling of throughput per step period
SIZING = {"per_conn_read": 512 << 10, "carry_cap": 1 << 20}


def get_pollers(port, n, prefill=200000):
    """``n`` clients polling Basic.Get (no-ack) on their own pre-filled queue while the
    load runs (bench/get_poller.py, a separate process): every answer is served inside a
    step (k_dequeue) without draining the pipeline.  Returns the process once its queues
    are filled; ``stop_pollers`` ends it and returns [(gets ok, gets empty, seconds)]."""
    import subprocess
    p = subprocess.Popen([sys.executable, os.path.join(os.path.dirname(os.path.abspath(__file__)), "get_poller.py"),
                          "--port", str(port), "--n", str(n), "--prefill", str(prefill)],
                         stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    line = p.stdout.readline()
    if line.strip() != "ready":
        p.kill()
        raise RuntimeError(f"get pollers failed to start: {line!r}")
    return p


def stop_pollers(p):
    import subprocess
    try:
        out, _ = p.communicate("", timeout=60)
    except subprocess.TimeoutExpired:
        p.kill()
        return []
    lines = [x for x in out.splitlines() if x.startswith("[")]
    return [tuple(x) for x in json.loads(lines[-1])] if lines else []


def churn_start(port, conn_threads=4, cons_threads=4, rpc_threads=0):
    """Connection open/close, consume/cancel and RPC-pattern churn in its own process
    (bench/churn_client.py)."""
    import subprocess
    p = subprocess.Popen([sys.executable, os.path.join(os.path.dirname(os.path.abspath(__file__)), "churn_client.py"),
                          "--port", str(port), "--conn-threads", str(conn_threads), "--cons-threads", str(cons_threads),
                          "--rpc-threads", str(rpc_threads)],
                         stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    line = p.stdout.readline()
    if line.strip() != "ready":
        p.kill()
        raise RuntimeError(f"churn client failed to start: {line!r}")
    return p


def churn_stop(p):
    import subprocess
    try:
        out, _ = p.communicate("", timeout=60)
    except subprocess.TimeoutExpired:
        p.kill()
        return {"error": "churn client did not stop"}
    lines = [x for x in out.splitlines() if x.startswith("{")]
    return json.loads(lines[-1]) if lines else {"error": "no churn result"}


def run_one(core, name, spec, io, io_threads, seconds, rate=0.0, lg_threads=12, store_dir=None, cons_threads=8,
            n_getters=0, churn=None, with_store=False):
    """with_store: a store (on disk, fsync on) attached even when the spec publishes nothing
    persistent: the broker then runs as a durable one (write-behind, held steps)."""
    from chanamq_amd.server.gpu_broker import GpuBroker
    persist = bool(spec.get("persistent")) or with_store
    plane = plane_for(dict(spec, persistent=persist))
    store = None
    if persist:
        store = core.Store()
        store.open(store_dir or tempfile.mkdtemp(prefix="cmq-gpu-store-"), True)
    bkw = dict(spec.get("_broker", {}))
    if persist and "persist_group_ms" in BROKER_CFG:
        bkw["persist_group_ms"] = BROKER_CFG["persist_group_ms"]
    if BROKER_CFG.get("confirm_read"):
        bkw["confirm_read"] = BROKER_CFG["confirm_read"]
    spec = {k: v for k, v in spec.items() if not k.startswith("_")}
    b = GpuBroker(plane, idle_step_ms=0.5, store=store, io=io, io_threads=io_threads,
                  per_conn_read=SIZING["per_conn_read"], fe_cfg=FE_CFG, **bkw).start()
    t0 = time.time()
    cpu0 = thread_cpu()
    timeline, done = [], [False]

    def sample():   # (s, live MB, blocked, published, delivered) every 100 ms
        while not done[0]:
            fs = getattr(b, "_fe_stats", None) or {}
            timeline.append((round(time.time() - t0, 2), round(fs.get("live_bytes", 0) / 2**20, 1), int(b.blocked),
                             fs.get("published", 0), fs.get("delivered", 0)))
            time.sleep(0.1)
    import threading
    smp = threading.Thread(target=sample, daemon=True)
    smp.start()
    gout, gproc = [], None
    if n_getters:
        gproc = get_pollers(b.port, n_getters)
    cproc, cout = None, None
    if churn:
        cproc = churn_start(b.port, *churn)
    st0 = {k: (dict(v) if isinstance(v, dict) else v) for k, v in b.stats.items()}
    try:
        if cproc is not None:
            cproc.stdin.write("go\n")
            cproc.stdin.flush()
        r = core.run_load(dict(port=b.port, seconds=seconds, warmup=1.0, queue=f"e2e.{name}",
                               exchange=f"e2e.x.{name}", threads=lg_threads, consumer_threads=cons_threads,
                               rate=rate, **spec))
    except Exception:   # what the broker still holds back when a client gives up on a reply
        try:
            b._sync_fe_stats()
            fs = getattr(b, "_fe_stats", None) or {}
            eng = getattr(plane, "eng", None)
            print(json.dumps({"diag": "load failed", "ctl_state": list(b.fe.ctl_state()) if b.fe else None,
                              "dl_state": [eng.dl_state(k) for k in range(4)] if eng is not None else None,
                              "lock": [b.lock.depth, b.lock.light, b.lock.paused_at],
                              "conns": [(c.id, c.state, len(c.out)) for c in list(b.conns.values())],
                              "conn_paused": [int(np.frombuffer(eng.download("conn_paused", 4 * c.id, 4), np.uint32)[0])
                                              for c in list(b.conns.values())] if eng is not None else None,
                              "held_steps": fs.get("held_steps"), "steps": fs.get("steps"),
                              "stats": {k: v for k, v in b.stats.items() if isinstance(v, (int, float, str))}}),
                  file=sys.stderr, flush=True)
            tr = list(b.ctl_trace or [])
            if tr:   # the connections whose last queue.declare has no queue.purge after it
                admin = sorted({e[1] for e in tr if e[2] != "flush" and e[3] == "queue.declare"
                                and str(e[6] or "").startswith("e2e.")})
                for cid in admin:
                    print(f"--- trace conn {cid}:", [e for e in tr if e[1] == cid][-40:], file=sys.stderr, flush=True)
            import traceback
            for tid, fr in sys._current_frames().items():   # where the control thread is
                st = traceback.format_stack(fr)
                if any("gpu_broker.py" in x for x in st):
                    print(f"--- thread {tid}\n" + "".join(st[-14:]), file=sys.stderr, flush=True)
        except Exception as e:   # noqa: BLE001
            print("diag failed:", e, file=sys.stderr, flush=True)
        raise
    finally:
        done[0] = True
        if gproc is not None:
            gout = stop_pollers(gproc)
        if cproc is not None:
            cout = churn_stop(cproc)
        st1 = {k: (dict(v) if isinstance(v, dict) else v) for k, v in b.stats.items()}
        smp.join()
        cpu1 = thread_cpu()
        after = {}
        try:   # the broker after the load: what stays live / pinned once every client is gone
            time.sleep(0.6)
            if b.fe is not None:
                b._sync_fe_stats()
                after = {k: b._fe_stats[k] for k in ("live_msgs", "live_bytes", "log_used")}
                with b.lock:
                    after["queue_depths"] = {q.name: plane.message_count(q.slot) for q in plane.queue_by_slot.values()
                                             if plane.message_count(q.slot)}
                    after["log_live_blocks"] = int((np.frombuffer(plane.eng.download("log_live"), np.int64) != 0).sum())
                    if after["live_msgs"]:
                        ent = np.dtype([("log_off", "<u8"), ("msg_id", "<u8"), ("ts", "<i8"), ("slot_bytes", "<u4"),
                                        ("body_len", "<u4"), ("body_off", "<u4"), ("props_len", "<u2"), ("ex_len", "u1"),
                                        ("rk_len", "u1"), ("refcnt", "<i4"), ("flags", "<u4"), ("pub_step", "<u4"),
                                        ("pad", "<u4"), ("href", "<u8")])
                        m = np.frombuffer(plane.eng.download("msgs"), ent)
                        free_top = plane.info["msg_max"] - after["live_msgs"]
                        fl = set(np.frombuffer(plane.eng.download("msg_free", 0, 4 * free_top), np.uint32).tolist())
                        queued = set()
                        for q in plane.queue_by_slot.values():
                            plane._refresh_ring(q)
                            h, t = plane._u64("q_head", q.slot), plane._u64("q_tail", q.slot)
                            raw = np.frombuffer(plane.eng.download("ring", q.ring_off * 16, q.capacity * 16), np.uint32)
                            for pos in range(h, t):
                                queued.add(int(raw[(pos & (q.capacity - 1)) * 4]))
                        live = [i for i in range(len(m)) if i not in fl and i not in queued]
                        after["queued_msgs"] = len(queued)
                        lm = m[live] if live else m[:1]
                        # where do the leaked indices still appear?  whole ring pool scan
                        top = plane._u64("ring_top", 0)
                        pool = np.frombuffer(plane.eng.download("ring", 0, top * 16), np.uint32).reshape(-1, 4)
                        lset = set(live)
                        hits = [i for i in range(len(pool)) if int(pool[i, 0]) in lset]
                        owner = {}
                        for q in plane.queue_by_slot.values():
                            owner.update({i: (q.name, q.ring_off, q.capacity) for i in range(q.ring_off, q.ring_off + q.capacity)})
                        after["leak_where"] = dict(n_hits=len(hits), in_live_ring=sum(1 for i in hits if i in owner),
                                                   sample=[(i, owner.get(i)) for i in hits[:8]])
                        after["leak_steps"] = sorted(set(lm["pub_step"].tolist()))[:40]
                        after["grow_log"] = getattr(b, "_grow_log", [])[:40]
                        after["leaked"] = dict(n=len(live), refcnt=sorted(set(lm["refcnt"].tolist()))[:8],
                                               pub_step=[int(lm["pub_step"].min()), int(lm["pub_step"].max())],
                                               steps_total=b._fe_stats["steps"], flags=sorted(set(lm["flags"].tolist())),
                                               body_len=sorted(set(lm["body_len"].tolist()))[:5])
        except Exception as e:   # diagnostics only
            after = {"error": repr(e)}
        b.stop()
        body_log = None
        if store is not None:
            body_log = store.body_stats() if hasattr(store, "body_stats") else None
            store.close()
    lc = getattr(plane, "last_counters", {}) or {}
    r["engine_host_s"] = {k: round(v, 4) for k, v in plane.eng.host_times(False).items()}
    r["after"] = after
    r["timeline"] = timeline
    r["thread_cpu_s"] = {k: round(cpu1[k] - cpu0.get(k, 0.0), 2) for k in cpu1 if cpu1[k] - cpu0.get(k, 0.0) > 0.05}
    st = dict(b.stats)
    fes = getattr(b, "_fe_stats", None) or {}
    r.update(name=name, io=io, io_threads=io_threads if io == "pipeline" else 1, loadgen_threads=lg_threads,
             rate_per_producer=rate, recv_msgs_per_s=r["received"] / r["elapsed"],
             sent_msgs_per_s=r["sent"] / r["elapsed"], confirmed_per_s=r["confirmed"] / r["elapsed"],
             wall_s=time.time() - t0, steps=st.get("steps"), spec=spec,
             front_end={k: fes.get(k) for k in ("steps", "idle_steps", "gather_segs", "io_phase_s", "wait_s",
                                                "submit_s", "rx_bytes", "tx_bytes", "held_steps", "published",
                                                "delivered", "routed", "dropped_nomem", "ring_full", "unroutable",
                                                "expired", "ctrl", "live_msgs", "live_bytes", "log_used",
                                                "h_period_us_log2", "h_io_us_log2", "h_submit_us_log2",
                                                "h_wait_us_log2", "max_period_s", "max_io_s", "max_wait_s")},
             flow_off_server=st.get("flow_off", 0),
             getters=(dict(n=n_getters, gets_ok=sum(g[0] for g in gout), gets_empty=sum(g[1] for g in gout),
                           gets_per_s=sum(g[0] + g[1] for g in gout) / max(1e-9, max((g[2] for g in gout), default=1)),
                           device_gets=st.get("device_gets", 0)) if n_getters else None),
             last_step={k: lc.get(k) for k in ("n_ring_full", "n_dropped_nomem")},
             churn=cout,
             control_sections=dict({k: st1.get(k, 0) - st0.get(k, 0) for k in ("pauses", "light_sections")},
                                   pause_why={k: v - (st0.get("pause_why") or {}).get(k, 0)
                                              for k, v in (st1.get("pause_why") or {}).items()}),
             store=getattr(b, "_pw_stats", None), body_log=body_log)
    del plane
    return r


def wal_soak(core, seconds, io_threads=4, lg_threads=12, cons_threads=8, rate=0.0):
    """BASELINE config 4 over TCP for ``seconds`` with the store on disk: the WAL size is
    sampled every second (background compaction keeps it bounded by the live rows), then
    the store is reopened (WAL replay) and a fresh plane recovers from it -- the restart
    cost after a long run."""
    from chanamq_amd.engine.persistence import GpuPersistence
    from chanamq_amd.server.gpu_broker import GpuBroker
    spec = {k: v for k, v in SPECS["config4_durable_4KB_confirms"].items() if not k.startswith("_")}
    d = tempfile.mkdtemp(prefix="cmq-wal-soak-")
    store = core.Store()
    store.open(d, True)
    plane = plane_for(spec)
    b = GpuBroker(plane, idle_step_ms=0.5, store=store, io="pipeline", io_threads=io_threads,
                  per_conn_read=SIZING["per_conn_read"]).start()
    samples, done = [], [False]
    t0 = time.time()

    def sample():
        while not done[0]:
            samples.append((round(time.time() - t0, 1), store.wal_bytes(), store.live_estimate(),
                            store.compact_stats()["runs"], store.body_stats()["disk_bytes"]))
            time.sleep(1.0)
    import threading
    th = threading.Thread(target=sample, daemon=True)
    th.start()
    try:
        r = core.run_load(dict(port=b.port, seconds=seconds, warmup=1.0, queue="soak.q", exchange="soak.x",
                               threads=lg_threads, consumer_threads=cons_threads, rate=rate, **spec))
    finally:
        done[0] = True
        th.join()
        b.stop()
    cs = store.compact_stats()
    wal_end = store.wal_bytes()
    rows = {t: store.row_count(t) for t in ("msgs", "queues", "queue_unacks")}
    body_log = store.body_stats()
    store.close()
    del plane
    t1 = time.perf_counter()
    st2 = core.Store()
    st2.open(d, True)
    replay_s = time.perf_counter() - t1
    plane2 = plane_for(spec)
    t2 = time.perf_counter()
    recovered = GpuPersistence(plane2, st2).recover(int(time.time() * 1000))
    recover_s = time.perf_counter() - t2
    st2.close()
    return dict(name="config4_wal_soak", seconds=seconds, recv_msgs_per_s=r["received"] / r["elapsed"],
                confirmed_per_s=r["confirmed"] / r["elapsed"], error=r["error"], wal_samples=samples,
                wal_end_bytes=wal_end, rows_at_end=rows, compactions=cs, reopen_replay_s=replay_s,
                recover_s=recover_s, recovered_msgs=recovered, body_log=body_log,
                body_bytes_written=getattr(b, "_pw_stats", {}).get("body_bytes"))


def run_sharded(core, name, spec, world, mode, seconds, rate=0.0, io_threads=2, lg_threads=12, cons_threads=8,
                churn=None):
    """The pipelined sharded server (server/sharded.py, ``world`` rank processes on this
    one GPU, shared-memory exchange): the topology is declared on rank 0 (its queues live
    there), producers attach to rank 1 (every publish crosses the per-step exchange) and
    consumers to rank 0 (``mode`` "local") or rank 1 (``mode`` "remote": every delivery
    travels back through a device link and every ack through the exchange)."""
    from chanamq_amd.parallel.launch import Launcher
    tmp = tempfile.mkdtemp(prefix="cmq-sharded-")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root)
    ln = Launcher(world, ["-m", "chanamq_amd.server.sharded", "--config", SMALL_CONF, "--plane", "gpu", "--port", "0", "--backend", "gloo",
                          "--info-dir", tmp, "--io-threads", str(io_threads), "--idle-step-ms", "0.5"]
                  + os.environ.get("CHANAMQ_SHARDED_ARGS", "").split(),
                  env=env).start()
    try:
        deadline = time.time() + 180
        while not all(os.path.exists(os.path.join(tmp, f"rank{r}.json")) for r in range(world)):
            if ln.poll() or time.time() > deadline:
                raise RuntimeError(f"sharded server did not come up: {ln.poll()}")
            time.sleep(0.2)
        ports = [json.load(open(os.path.join(tmp, f"rank{r}.json")))["port"] for r in range(world)]
        spec = {k: v for k, v in spec.items() if not k.startswith("_")}
        t0 = time.time()
        cproc, cout = None, None
        if churn:   # on the consumers' rank: its queues live there, its control ops stay local
            cproc = churn_start(ports[0], *churn)
            cproc.stdin.write("go\n")
            cproc.stdin.flush()
        try:
            r = core.run_load(dict(port=ports[0], consumer_port=ports[0] if mode == "local" else ports[1 % world],
                                   producer_port=ports[1 % world], seconds=seconds, warmup=1.0,
                                   queue=f"e2e.{name}", exchange=f"e2e.x.{name}", threads=lg_threads,
                                   consumer_threads=cons_threads, rate=rate, **spec))
        finally:
            if cproc is not None:
                cout = churn_stop(cproc)
        time.sleep(0.7)
        ranks = [json.load(open(os.path.join(tmp, f"rank{k}.json"))) for k in range(world)]
    finally:
        ln.stop()
    r["churn"] = cout
    r.update(name=name, io="pipeline-sharded", world=world, consumers_on=mode, io_threads=io_threads,
             rate_per_producer=rate, recv_msgs_per_s=r["received"] / r["elapsed"],
             sent_msgs_per_s=r["sent"] / r["elapsed"], confirmed_per_s=r["confirmed"] / r["elapsed"],
             wall_s=time.time() - t0, spec=spec,
             ranks=[{"rank": k["rank"], "front_end": {x: k["front_end"].get(x) for x in
                                                      ("steps", "idle_steps", "xchg_steps", "syncs", "xfails",
                                                       "flush_steps", "xchg_s", "submit_s", "io_phase_s", "wait_s",
                                                       "published", "delivered", "held_steps")},
                     "control_sections": {x: k["stats"].get(x) for x in ("pauses", "light_sections", "pause_why")}}
                    for k in ranks])
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--out", default="")
    ap.add_argument("--only", default="")
    ap.add_argument("--io", default="pipeline", help="comma list of front ends: pipeline,native")
    ap.add_argument("--io-threads", default="4", help="comma list (pipeline front end)")
    ap.add_argument("--loadgen-threads", type=int, default=12)
    ap.add_argument("--consumer-threads", type=int, default=8, help="of the load generator's threads")
    ap.add_argument("--wblock-high", type=int, default=0, help="front end egress back-pressure high watermark (B)")
    ap.add_argument("--per-conn-read", type=int, default=512 << 10, help="bytes per connection per step")
    ap.add_argument("--carry-cap", type=int, default=1 << 20, help="device carry per connection (>= 2x per-conn-read)")
    ap.add_argument("--rates", default="", help="comma list of aggregate publish rates (msgs/s) to run paced")
    ap.add_argument("--paced", type=float, default=0.5,
                    help="re-run each spec with producers paced at this fraction of the measured rate (0 = off)")
    ap.add_argument("--wal-soak", type=float, default=0,
                    help="run config 4 for this many seconds with the store on disk, sample the WAL, "
                         "then time the reopen + recovery")
    ap.add_argument("--sharded", type=int, default=0,
                    help="N > 1: the pipelined sharded server with N ranks on this GPU (producers on rank 1, "
                         "consumers on rank 0 and then on rank 1 through device links)")
    ap.add_argument("--spill-bytes", type=int, default=8 << 30, help="host spill ring of the bench plane (0 = off)")
    ap.add_argument("--confirm-read", type=int, default=0,
                    help="bytes per confirm-mode connection per step (0 = the broker default, 128 KiB)")
    ap.add_argument("--persist-group-ms", type=float, default=2.0,
                    help="durable specs: a group commit waits until its oldest batch is this old")
    ap.add_argument("--churn", action="store_true",
                    help="paced runs again next to connection open/close and consume/cancel churn "
                         "(bench/churn_client.py): delivered rate and latency with and without it")
    ap.add_argument("--churn-threads", default="4,4,0", help="connection,consumer,rpc churn threads")
    ap.add_argument("--churn-store", action="store_true",
                    help="--churn: the broker runs with a store on disk (fsync on), i.e. as a durable broker")
    ap.add_argument("--getters", type=int, default=0,
                    help="also run each spec with this many Basic.Get pollers on pre-filled queues (the load's "
                         "throughput with and without them, and the gets/s)")
    ap.add_argument("--egress-ref", type=int, default=1,
                    help="1: the front end sends delivered bodies from the host ingress arenas (egress by "
                         "reference); 0: every delivered body comes back over PCIe in the egress bytes")
    ap.add_argument("--plane-cfg", default='{"copy_engine": 3, "overlap": 0, "h2d_hsa": 1}',
                    help="JSON engine settings for the server plane; default: the single-GPU server's step "
                         "pipeline (SDMA egress, one graph, ingress through HSA -- chana.mq.gpu.copy-engine / "
                         "overlap / h2d-hsa); '{}': the engine's defaults (blit egress, overlapped ingest)")
    ap.add_argument("--with-store", action="store_true",
                    help="every run with a store on disk attached (a durable broker)")
    args = ap.parse_args()
    FE_CFG["egress_ref"] = bool(args.egress_ref)
    BROKER_CFG["persist_group_ms"] = args.persist_group_ms
    BROKER_CFG["confirm_read"] = args.confirm_read
    SIZING["spill_bytes"] = args.spill_bytes
    if args.plane_cfg:
        SIZING["plane_cfg"] = json.loads(args.plane_cfg)
    SIZING.update(per_conn_read=args.per_conn_read, carry_cap=max(args.carry_cap, 2 * args.per_conn_read))
    if args.wblock_high:
        FE_CFG.update(wblock_high=args.wblock_high, wblock_low=args.wblock_high // 4)
    core = load()
    results = []
    if args.wal_soak > 0:
        import torch  # noqa: F401
        r = wal_soak(core, args.wal_soak, io_threads=int(args.io_threads.split(",")[0]))
        print(json.dumps({k: v for k, v in r.items() if k != "wal_samples"}), flush=True)
        if args.out:
            with open(args.out, "w") as f:
                json.dump(r, f, indent=1)
        return
    if args.sharded > 1:
        keys = ("name", "world", "consumers_on", "recv_msgs_per_s", "sent_msgs_per_s", "confirmed_per_s", "p50_us",
                "p99_us", "error", "ranks")
        for name, spec in SPECS.items():
            if args.only and args.only not in name:
                continue
            for mode in ("local", "remote"):
                r = run_sharded(core, name, spec, args.sharded, mode, args.seconds, io_threads=int(args.io_threads.split(",")[0]),
                                lg_threads=args.loadgen_threads, cons_threads=args.consumer_threads)
                results.append(r)
                print(json.dumps({k: r.get(k) for k in keys}), flush=True)
                if args.paced > 0 and r["recv_msgs_per_s"] > 0 and not r["error"]:
                    rate = args.paced * r["recv_msgs_per_s"] / max(1, spec.get("producers", 1))
                    rp = run_sharded(core, name, spec, args.sharded, mode, args.seconds, rate=rate,
                                     io_threads=int(args.io_threads.split(",")[0]), lg_threads=args.loadgen_threads,
                                     cons_threads=args.consumer_threads)
                    rp["paced_fraction"] = args.paced
                    results.append(rp)
                    print(json.dumps({k: rp.get(k) for k in keys + ("rate_per_producer", "p95_us")}), flush=True)
                    if args.churn and mode == "local":
                        ct = tuple(int(x) for x in args.churn_threads.split(","))
                        rc = run_sharded(core, name, spec, args.sharded, mode, args.seconds, rate=rate,
                                         io_threads=int(args.io_threads.split(",")[0]), lg_threads=args.loadgen_threads,
                                         cons_threads=args.consumer_threads, churn=ct)
                        rc["paced_fraction"] = args.paced
                        rc["delivered_vs_no_churn"] = rc["recv_msgs_per_s"] / max(1e-9, rp["recv_msgs_per_s"])
                        results.append(rc)
                        print(json.dumps({k: rc.get(k) for k in keys + ("rate_per_producer", "p95_us",
                                                                        "delivered_vs_no_churn", "churn")}), flush=True)
        if args.out:
            with open(args.out, "w") as f:
                json.dump({"meta": {"transport": "loopback TCP", "data_plane": f"HIP gfx950, {args.sharded} ranks on 1 GPU",
                                    "exchange": "host shared memory (RCCL needs one GPU per rank)",
                                    "seconds": args.seconds}, "results": results}, f, indent=1)
        return
    import torch  # noqa: F401  (HIP runtime up before the first plane)
    for name, spec in SPECS.items():
        if args.only and args.only not in name:
            continue
        for io in args.io.split(","):
            for nt in ([int(x) for x in args.io_threads.split(",")] if io == "pipeline" else [1]):
                r = run_one(core, name, spec, io, nt, args.seconds, lg_threads=args.loadgen_threads,
                               cons_threads=args.consumer_threads, with_store=args.with_store)
                results.append(r)
                print(json.dumps({k: r[k] for k in ("name", "io", "io_threads", "recv_msgs_per_s", "sent_msgs_per_s",
                                                    "confirmed_per_s", "p50_us", "p99_us", "error", "redelivered",
                                                    "requeued", "flow_off", "flow_off_server", "front_end",
                                                    "store", "thread_cpu_s", "cpu_consumers_s",
                                                    "cpu_producers_s", "engine_host_s")}),
                      flush=True)
                if args.getters:
                    rg = run_one(core, name, spec, io, nt, args.seconds, lg_threads=args.loadgen_threads,
                                 cons_threads=args.consumer_threads, n_getters=args.getters)
                    rg["with_getters"] = args.getters
                    results.append(rg)
                    print(json.dumps({k: rg[k] for k in ("name", "io_threads", "recv_msgs_per_s", "sent_msgs_per_s",
                                                         "p50_us", "p99_us", "getters", "error")}), flush=True)
                for agg in [float(x) for x in args.rates.split(",") if x]:
                    rr = run_one(core, name, spec, io, nt, args.seconds, rate=agg / max(1, spec.get("producers", 1)),
                                 lg_threads=args.loadgen_threads, cons_threads=args.consumer_threads)
                    rr["aggregate_rate"] = agg
                    results.append(rr)
                    print(json.dumps({k: rr[k] for k in ("name", "io_threads", "aggregate_rate", "sent_msgs_per_s",
                                                         "recv_msgs_per_s", "p50_us", "p99_us", "thread_cpu_s",
                                                         "cpu_consumers_s", "cpu_producers_s", "error")}), flush=True)
                if args.paced > 0 and r["recv_msgs_per_s"] > 0 and not r["error"]:
                    rate = args.paced * r["recv_msgs_per_s"] / max(1, spec.get("producers", 1))
                    if spec.get("exchange_type") == "fanout":   # deliveries = publishes x queues
                        rate /= max(1, spec.get("queues", 1))
                    rp = run_one(core, name, spec, io, nt, args.seconds, rate=rate, lg_threads=args.loadgen_threads,
                               cons_threads=args.consumer_threads, with_store=args.with_store)
                    rp["paced_fraction"] = args.paced
                    results.append(rp)
                    print(json.dumps({k: rp[k] for k in ("name", "io", "io_threads", "rate_per_producer",
                                                         "recv_msgs_per_s", "p50_us", "p95_us", "p99_us",
                                                         "error", "control_sections")}), flush=True)
                    if args.churn:
                        ct = tuple(int(x) for x in args.churn_threads.split(","))
                        if args.churn_store:   # the no-churn reference with the same store attached
                            rp = run_one(core, name, spec, io, nt, args.seconds, rate=rate,
                                         lg_threads=args.loadgen_threads, cons_threads=args.consumer_threads,
                                         with_store=True)
                            rp["paced_fraction"] = args.paced
                            rp["with_store"] = True
                            results.append(rp)
                            print(json.dumps({k: rp[k] for k in ("name", "io_threads", "recv_msgs_per_s", "p50_us",
                                                                 "p99_us", "error", "control_sections")}), flush=True)
                        rc = run_one(core, name, spec, io, nt, args.seconds, rate=rate, lg_threads=args.loadgen_threads,
                                     cons_threads=args.consumer_threads, churn=ct, with_store=args.churn_store)
                        rc["with_store"] = args.churn_store
                        rc["paced_fraction"] = args.paced
                        rc["delivered_vs_no_churn"] = rc["recv_msgs_per_s"] / max(1e-9, rp["recv_msgs_per_s"])
                        results.append(rc)
                        print(json.dumps({k: rc[k] for k in ("name", "io_threads", "rate_per_producer", "recv_msgs_per_s",
                                                             "delivered_vs_no_churn", "p50_us", "p95_us", "p99_us",
                                                             "error", "churn", "control_sections")}), flush=True)
    if args.out:
        import platform
        with open(args.out, "w") as f:
            json.dump({"meta": {"transport": "loopback TCP", "data_plane": "HIP gfx950 (1 GPU)",
                                "host_cpus_visible": os.cpu_count(), "machine": platform.machine(),
                                "latency": "publish->deliver from the send timestamp in each body (steady clock)",
                                "seconds": args.seconds, "warmup_s": 1.0},
                       "results": results}, f, indent=1)


if __name__ == "__main__":
    main()
