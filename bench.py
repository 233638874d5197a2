#!/usr/bin/env python3
"""Headline benchmark: msgs/sec (whole node) + p50 publish->deliver latency, 1 KB payload.

Workload = BASELINE.json config 2 per GPU ("1 topic exchange, 16 bound queues, 1 KB msgs,
auto-ack"), weak-scaled: each rank (one MI355X) owns 16 queues and their consumers and
serves 256 producer connections.  With N>1 the ranks form ONE sharded broker: exchanges
and bindings are replicated, every producer publishes uniformly over all 16*N queues of
the node, so (N-1)/N of the messages are routed on the ingress GPU and shipped to the
owning GPU by the per-step RCCL all-to-all (parallel/exchange.py) before they are
enqueued and delivered there (``--mode independent`` = N unconnected shards).
Producers are synthetic AMQP connections whose
wire bytes (Basic.Publish method + content header + 1 KB body frame) are pre-rendered
into a pinned ingress pool and handed to the data plane in TCP-read-sized chunks that
split frames at arbitrary offsets.  One timed step = the full broker hot path on the
GPU: H2D of the step's ingress bytes, frame scan, command assembly, publish decode,
topic routing (MFMA prefilter + exact matcher), message store, queue enqueue, dequeue
to consumers, delivery tags, Basic.Deliver rendering into host-mapped egress memory,
auto-ack release — nothing skipped.

python bench.py [--gpus N --steps K --warmup W]   (N>1: launched by torch.distributed.run)
"""

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

METRIC = "msgs/sec (whole node) + p50 publish→deliver latency, 1 KB payload, 1/2/4/8 GPUs"


def build_workload(dp, rank, producers, queues, body, chunk, blocks, cons_base, shards=1, kind="topic", consume=True,
                   qcap=None):
    """``shards`` > 1: the replicated topology of a sharded broker (every rank declares
    every queue; queue bench.q.{r}.{i} is placed on rank r and consumed there).
    kind "topic" = config 2 (``queues`` per rank, one key pattern each); "fanout" =
    config 3 (every publish goes to every queue of the node); "storm" = config 5 (direct,
    manual-ack consumers that ack everything each step and nack-requeue everything every
    4th step)."""
    from chanamq_amd.engine.layout import SEG_IN
    from chanamq_amd.engine.traffic import even_split, publish_stream

    vh = "AMQ.DEFAULT"
    xname = {"topic": "bench.topic", "fanout": "bench.fanout", "storm": "bench.direct"}[kind]
    dp.declare_exchange(vh, xname, "direct" if kind == "storm" else kind)
    owners = range(shards) if shards > 1 else [rank]
    for r in owners:
        for i in range(queues):
            qn = f"bench.q.{r}.{i}"
            if shards > 1:
                dp.shard_map.place(vh, qn, r)
            dp.declare_queue(vh, qn, capacity=qcap or (1 << 14 if kind == "fanout" else 1 << 20))
            key = {"topic": f"bench.{r}.{i}.*", "fanout": "", "storm": f"bench.{r}.{i}"}[kind]
            dp.bind(vh, qn, xname, key)
    for p in range(producers):
        dp.open_connection(p, vh)
        dp.open_channel(p, 1)
    for i in range(queues):
        c = cons_base + i
        dp.open_connection(c, vh)
        dp.open_channel(c, 1)
        if kind == "storm":
            dp.qos(c, 1, prefetch_count=512)
        if consume:
            dp.consume(c, 1, vh, f"bench.q.{rank}.{i}", f"ctag-{i}", no_ack=kind != "storm")
    # one message on the wire is ~1.08 KB; each producer gets `blocks` chunks of ~chunk bytes
    probe = publish_stream(1, xname, lambda i: f"bench.{rank}.0.x0", body)
    per_prod = max(1, (chunk * blocks) // len(probe))
    streams = []
    nq = queues * len(owners)
    for p in range(producers):
        rng_q = np.random.default_rng(1000 + rank * 7919 + p).integers(0, nq, size=per_prod)
        if kind == "storm":
            keyf = (lambda i, r=rng_q: f"bench.{owners[r[i] // queues]}.{r[i] % queues}")
        else:
            keyf = (lambda i, r=rng_q: f"bench.{owners[r[i] // queues]}.{r[i] % queues}.x{i % 10}")
        s = publish_stream(per_prod, xname, keyf, body, seed=p)
        streams.append(even_split(s, blocks))
    # block-major pinned pool: block b = chunk b of every producer, 16-B aligned
    sizes = [[len(streams[p][b]) for p in range(producers)] for b in range(blocks)]
    ctl = b""
    if kind == "storm":   # consumer frames: ack-all, nack-all-requeue (delivery-tag 0 + multiple)
        from chanamq_amd.engine.traffic import ack_frame
        from chanamq_amd.protocol.codec import Method, render_command
        ack = ack_frame(1, 0, multiple=True)
        nack = render_command(1, Method("basic.nack", delivery_tag=0, multiple=True, requeue=True))
        ctl = ack + b"\0" * ((-len(ack)) % 16) + nack
        ctl += b"\0" * ((-len(ctl)) % 16)
    # each block = the producers' chunks, then the consumer control frames (storm)
    data_len = [sum((n + 15) & ~15 for n in row) for row in sizes]
    block_len = [n + len(ctl) for n in data_len]
    total = sum(block_len)
    pool = dp.mod.alloc_pinned(total + 64)
    segs, offs = [], []
    off = 0
    for b in range(blocks):
        offs.append(off)
        sg = np.zeros(producers, SEG_IN)
        rel = 0
        for p in range(producers):
            data = streams[p][b]
            pool[off + rel:off + rel + len(data)] = np.frombuffer(data, np.uint8)
            sg[p] = (p, len(data), rel)
            rel += (len(data) + 15) & ~15
        segs.append(sg)
        if ctl:
            pool[off + data_len[b]:off + data_len[b] + len(ctl)] = np.frombuffer(ctl, np.uint8)
        off += block_len[b]
    msgs_per_step = per_prod * producers / blocks
    extra = None
    if kind == "storm":   # per-step consumer segments, offsets relative to each block's base
        extra = {}
        nack_rel = len(ack) + ((-len(ack)) % 16)
        for name, o, ln in (("ack", 0, len(ack)), ("nack", nack_rel, len(nack))):
            extra[name] = [np.array([(cons_base + i, ln, data_len[b] + o) for i in range(queues)], SEG_IN)
                           for b in range(blocks)]
    return pool, segs, offs, block_len, msgs_per_step, len(probe), extra


def verify_egress(dp, base, pool_len, tickets):
    """Egress by reference, checked outside the timed window on finished steps: every
    gather entry points into the retained ingress pool, and the spliced wire bytes of every
    connection parse as complete AMQP frames and commands (a missing or misplaced body breaks
    the frame-end markers).  Returns the number of Basic.Deliver commands checked."""
    from chanamq_amd.engine.layout import EGRESS_REF
    from chanamq_amd.protocol.codec import CommandAssembler, FrameParser
    checked = 0
    if True:
        for t in tickets:
            c = dp.eng.counters(t[0])
            eg, co = dp.host_egress(t)
            if c["n_ref"]:
                raw = dp._egress[t[3]]
                tab = raw[c["gath_off"]:c["gath_off"] + 16 * c["n_deliv"]].view(EGRESS_REF)
                r = tab[tab["len"] > 0]
                assert ((r["src"] >= base) & (r["src"] + r["len"] <= base + pool_len)).all(), "gather outside pool"
                assert (np.diff(tab["dst"].astype(np.int64)) >= 0).all(), "gather table not monotone"
            for conn in np.nonzero(co["len"])[0]:
                o, n = int(co["off"][conn]), int(co["len"][conn])
                fp, ca = FrameParser(), CommandAssembler()
                for f in fp.feed(bytes(eg[o:o + n])):
                    cmd = ca.feed(f)
                    if cmd is not None and cmd.method.name == "basic.deliver":
                        checked += 1
    return checked


def setup_native_exchange(args, cfg, GpuDataPlane, dist, backend, local, rank, world):
    """The sharded plane on the engine's native exchange, as the sharded server builds it
    (server/sharded.py): rank 0 draws the RCCL unique id and names the shared-memory
    segments, every rank receives them over the launcher's process group.  Returns None on
    every rank when any rank could not set it up (all ranks then use the torch exchange)."""
    import uuid

    import torch
    dp, err = None, None
    # (CHANAMQ_BENCH_XCHG=rccl under gloo: the RCCL code path through CHANAMQ_RCCL_LIB, the
    # tests' one-GPU stand-in -- a rehearsal, not a scaling number)
    kind = os.environ.get("CHANAMQ_BENCH_XCHG") or ("rccl" if backend == "nccl" else "shm")
    try:
        dp = GpuDataPlane(device=local, worker=rank, world=world, rank=rank, native_xchg=1, **cfg)
        names = [None]
        if rank == 0:
            tag = f"cmq-bench-{os.getpid()}-{uuid.uuid4().hex[:10]}"
            names = [{"uid": dp.xchg_unique_id() if kind == "rccl" else None, "shm": tag}]
        dist.broadcast_object_list(names, src=0)
        nm = names[0]
        if kind == "rccl":
            dp.xchg_setup("rccl", nm["uid"], list(range(world)), args.xchg_timeout_ms, counts_shm=nm["shm"] + "-c",
                          async_x=bool(args.async_x))
        else:
            dp.xchg_setup("shm", nm["shm"], list(range(world)), args.xchg_timeout_ms, async_x=bool(args.async_x))
    except Exception as e:   # noqa: BLE001 - reported, then agreed on below
        err = e
    bad = torch.tensor([1.0 if err is not None else 0.0], device="cuda" if backend == "nccl" else "cpu")
    dist.all_reduce(bad, op=dist.ReduceOp.MAX)
    if bad.item() > 0:
        if err is not None:
            print(f"rank {rank}: native exchange setup failed: {err!r}", file=sys.stderr, flush=True)
        del dp
        return None
    return dp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--producers", type=int, default=256)
    ap.add_argument("--queues", type=int, default=16)
    ap.add_argument("--body", type=int, default=1024)
    ap.add_argument("--chunk", type=int, default=49152,
                    help="bytes per producer per step (TCP read); 49152: 35-37.5 M msgs/s at p50 0.82-0.94 ms at K=20 "
                         "(65536: ~38 M at p50 1.08 ms, but box-to-box outliers; 32768: ~30 M at 0.73 ms; "
                         "profiles/r4_summary.md)")
    ap.add_argument("--blocks", type=int, default=8)
    ap.add_argument("--soak-s", type=float, default=2.0,
                    help="after the timed steps (and the result line), keep stepping untimed for this long so "
                         "an external GPU-utilisation sampler sees the workload (0 = off)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--overlap", type=int, default=0, choices=[0, 1],
                    help="1: a step's ingest half on its own high-priority stream (it may run beside the "
                         "previous step's routing half); 0 (default): the whole step as one graph on one "
                         "stream (no cross-queue hand-off between the halves; measured equal throughput, "
                         "p50 0.85 vs 1.10 ms at 49152, profiles/r5_fs1, r5_split)")
    ap.add_argument("--parities", type=int, default=2, choices=[2, 3],
                    help="per-step IO sets of the engine (single GPU, --overlap 0): 2 (default) = double buffering; "
                         "3 = the next step is submitted once step t-2 is collected -- measured the same step period "
                         "at p50 0.79 vs 0.54 ms (profiles/r6_u): the period is the GPU's, not the host's")
    ap.add_argument("--h2d-alt", type=int, default=0, choices=[0, 1],
                    help="1: odd steps' ingress H2D on a second stream (single GPU, --overlap 0)")
    ap.add_argument("--h2d-hsa", type=int, default=1, choices=[0, 1],
                    help="1 (default): the ingress payload copy queued on an SDMA engine through HSA and waited "
                         "for on the device (k_h2d_wait) -- no HIP marker / cross-queue barrier between two "
                         "steps' copies, which run back to back (measured 46.3 vs 43.4 M msgs/s, p50 0.50 vs "
                         "0.54 ms, profiles/r6_h1); 0: hipMemcpyAsync + event + stream wait (single GPU, "
                         "--overlap 0, --copy-engine sdma)")
    ap.add_argument("--h2d-at-wait", type=int, default=1, choices=[0, 1],
                    help="1: queue the next step's payload H2D right after the wait on step t-1's kernels "
                         "(its latency clock starts there); 0: at its submit")
    ap.add_argument("--loop", choices=["poll", "block"], default="block",
                    help="host loop: poll = submit as soon as a parity frees and stamp each egress when it "
                         "lands (non-blocking queries); block = submit / prefetch / wait egress t-2 / finish t-1")
    ap.add_argument("--egress-gate", type=int, default=1, choices=[0, 1],
                    help="1: each step's egress D2H is queued on the SDMA engine at launch and started by the "
                         "step's last kernel (no host round trip); 0: issued by the host once it saw the step finish")
    ap.add_argument("--copy-engine", choices=["kernel", "nocu", "blit", "sdma"], default="sdma",
                    help="egress D2H: an SDMA engine other than the ingress H2D's (default: H2D and D2H "
                         "overlap at ~47 GB/s each, bench/pcie_probe.hip), the runtime blit kernel (holds CUs "
                         "for the whole transfer), the runtime's NoCU request, or our copy kernel")
    ap.add_argument("--copy-wgs", type=int, default=16)
    ap.add_argument("--sdma-split", type=int, default=1,
                    help="--copy-engine sdma: egress D2H of >= 2 MB split over this many SDMA engines (1 or 2)")
    ap.add_argument("--sdma-engine", type=int, default=-1,
                    help="--copy-engine sdma: SDMA engine for the egress D2H (-1 = highest available)")
    ap.add_argument("--workload", choices=["topic", "fanout", "storm"], default="topic",
                    help="topic = BASELINE config 2 (default, the headline); fanout = config 3 "
                         "(--queues is then the node total, default 1024, with small publish batches)")
    ap.add_argument("--exchange-lag", type=int, choices=[0, 1], default=1,
                    help="N>1: 1 = pipelined all-to-all (phase B imports the previous step's exchange, "
                         "the collective overlaps the next step); 0 = synchronous")
    ap.add_argument("--mode", choices=["sharded", "independent"], default="sharded",
                    help="N>1: one sharded broker (cross-GPU routing over RCCL) or N unconnected shards")
    ap.add_argument("--prefetch", type=int, default=0, choices=[0, 1, 2],
                    help="N: keep the ingress H2D of the next N steps queued (submitted step t -> t+1..t+N; "
                         "the copy engine never idles between steps; a step's latency clock starts when its "
                         "bytes are queued); 0 (default): H2D at submit.  With the whole step on one stream "
                         "0 is best at the default step: K=200 38.8 M msgs/s at p50 0.85 ms vs 37.5 M at "
                         "1.12 ms with 1 (profiles/r5_split); at 32768 B 1 is faster (31 vs 27 M)")
    ap.add_argument("--xchg", choices=["native", "torch"], default="native",
                    help="N>1 sharded: the engine's own exchange -- grouped RCCL send/recv on its exchange "
                         "stream, counts through host shared memory (the code the sharded server runs; "
                         "CHANAMQ_BENCH_BACKEND=gloo: the shared-memory backend) -- or torch.distributed "
                         "all_to_all_single (parallel/exchange.py)")
    ap.add_argument("--xchg-timeout-ms", type=int, default=30000)
    ap.add_argument("--egress-ref", type=int, default=1, choices=[0, 1],
                    help="1 (default): egress by reference -- a delivery whose body arrived in the same step's "
                         "ingress payload is rendered without it and the host sends the body from that payload "
                         "(the pinned pool block, unchanged until the block is submitted again 8 steps later), so "
                         "bodies cross PCIe once; the D2H carries the frames + a gather table.  0: every body "
                         "rendered into HBM egress and copied D2H")
    ap.add_argument("--async-x", type=int, default=0,
                    help="1: native exchange on the engine's exchange thread, phase B waiting on the device "
                         "(default 0: the stepper runs each exchange itself; profiles/r5_summary.md)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:   # lockstep exchange steps: the blocking loop (every rank submits in step)
        args.loop = "block"
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    dist = None
    # CHANAMQ_BENCH_BACKEND=gloo rehearses the multi-rank path on fewer GPUs (ranks share
    # devices, exchange staged through the host); the real run uses RCCL ("nccl")
    backend = os.environ.get("CHANAMQ_BENCH_BACKEND", "nccl")
    if world > 1:
        import torch.distributed as dist
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    from chanamq_amd.engine.dataplane import GpuDataPlane

    fan = args.workload == "fanout"
    storm = args.workload == "storm"
    if fan and args.queues == 16:
        args.queues = 1024
    if fan and args.producers == 256:
        args.producers, args.chunk = 16, 4096
    if storm and args.queues == 16:     # config 5: 64 producers x 64 manual-ack consumers per GPU
        args.queues = 64
    if storm and args.producers == 256:
        args.producers, args.chunk = 64, 16384
    shards = world if (world > 1 and args.mode == "sharded") else 1
    P = args.producers
    Q = max(1, args.queues // shards) if fan else args.queues    # queues per rank
    qtot = Q * shards
    qcap = (1 << 20) if not fan else (1 << 14)
    cfg = dict(c_max=max(1024, P + Q + 1), chpc=4, q_max=max(64, qtot + 64), cons_max=max(1024, Q + 16),
               seg_max=max(1024, P + Q), cmd_max=1 << 17, deliv_max=(1 << 16) if not fan else (1 << 18),
               msg_max=1 << 22, ucap=4096, deliver_cap=8192,
               ingress_cap=max(32 << 20, P * args.chunk + (4 << 20)),
               egress_cap=(128 << 20) if not fan else (320 << 20),
               log_bytes=16 << 30, ring_pool=Q * qcap + qtot + 1024, tb_max=max(64, qtot) if not fan else 64,
               fan_max=max(1 << 20, qtot * 2), carry_cap=256 << 10, graph=0 if args.no_graph else 1,
               copy_engine={"blit": 0, "nocu": 1, "kernel": 2, "sdma": 3}[args.copy_engine], copy_wgs=args.copy_wgs, sdma_engine=args.sdma_engine,
               sdma_split=args.sdma_split, egress_gate=args.egress_gate, overlap=args.overlap, parities=args.parities,
               h2d_alt=args.h2d_alt, h2d_hsa=args.h2d_hsa,
               egress_ref=0 if args.egress_ref else -1)
    native = shards > 1 and args.xchg == "native"
    if native:
        dp = setup_native_exchange(args, cfg, GpuDataPlane, dist, backend, local, rank, world)
        if dp is None:   # refused on some rank (e.g. librccl): every rank falls back together
            native = False
            args.xchg = "torch (native exchange setup failed)"
    if shards > 1 and not native:
        from chanamq_amd.parallel.exchange import Exchanger
        dp = GpuDataPlane(device=local, worker=rank, world=world, rank=rank, exchanger=Exchanger(),
                          exchange_lag=args.exchange_lag, **cfg)
    elif shards == 1:
        dp = GpuDataPlane(device=local, worker=rank, **cfg)
    pool, segs, offs, blens, mps, msg_bytes, extra = build_workload(dp, rank, P, Q, args.body, args.chunk,
                                                                    args.blocks, cons_base=P, shards=shards,
                                                                    kind=args.workload)
    npar = dp.info.get("parities", 2)   # steps in flight before the host waits for the oldest
    flow_high = 1 << 30      # storm: producers pause (Channel.Flow) above 1 GiB of stored bodies
    flow = {"paused": False, "paused_steps": 0, "requeued": 0}
    base = pool.ctypes.data
    step_i = 0
    submit = dp.submit_lockstep if native else dp.submit_raw

    sub_t = {}      # step index -> host time its ingress was handed to the GPU (submit / prefetch)
    slow = {"ms": 0.0}   # the timed window's slowest loop iteration: submit / prefetch / egress / finish
    phases = []          # every timed iteration's phases (ms): submit, prefetch, egress wait, finish
    pre = set()     # steps whose payload H2D is already queued (prefetch)
    lat_w = []      # (publish->deliver seconds, deliveries) of the timed steps
    wire, nref = [0], [0]

    def run(n, measure=False):
        # software pipeline, 3 steps in flight: H2D(t+1) || kernels(t) || D2H(t-1);
        # the host consumes step t-1's results/egress while the GPU runs step t
        nonlocal step_i
        dl = pb = 0
        hist = np.zeros(32, np.int64)
        eg = 0
        wire[0] = 0
        pending = []    # (ticket, step index)
        waited = []     # the step whose kernels were waited for, not collected yet
        done = []
        lat_of = {}     # step index -> its lat_hist (deliveries by publish-step lag)

        def account(r, s):
            nonlocal dl, pb, eg
            c = r.counters
            dl += c["n_deliv"]
            pb += c["n_pubs"]
            eg += c["egress_bytes"]
            # bytes on the wire: the rendered frames + the referenced bodies (not the table)
            tab = 16 * c["n_deliv"] if c["n_ref"] else 0
            wire[0] += c["egress_bytes"] - tab + c["ref_bytes"]
            nref[0] += c["n_ref"]
            lh = np.array(c["lat_hist"], np.int64)
            hist[:] += lh
            lat_of[s] = lh
            if storm:
                flow["requeued"] += c["n_requeue"]
                flow["paused"] = c["live_bytes"] > flow_high

        def ready(s):
            # measured latency: a delivery rendered in step s whose message was published
            # k steps earlier waited from that step's submit until s's egress was in host
            # memory (bin 31 = 31 or more steps: counted as 31)
            t = time.perf_counter()
            lh = lat_of.pop(s, None)
            if measure and lh is not None:
                for k in np.nonzero(lh)[0]:
                    t0 = sub_t.get(s - int(k))
                    if t0 is not None:
                        lat_w.append((t - t0, int(lh[k])))

        end = step_i + n

        def submit_next():
            nonlocal step_i
            b = step_i % args.blocks
            if step_i not in pre:   # (a prefetched step's clock started when its bytes were queued)
                sub_t[step_i] = time.perf_counter()
            pre.discard(step_i)
            if storm:   # ack-all each step, nack-all-requeue every 4th: a redelivery storm
                cs = extra["nack" if step_i % 4 == 3 else "ack"][b]
                if flow["paused"]:
                    flow["paused_steps"] += 1
                    sg = cs
                else:
                    sg = np.concatenate([segs[b], cs])
            else:
                sg = segs[b]
            t = submit(sg, base + offs[b], blens[b])
            s = step_i
            step_i += 1
            nxt = max(step_i, max(pre) + 1 if pre else step_i)
            while args.prefetch and nxt < min(step_i + args.prefetch, end):
                nb = nxt % args.blocks
                sub_t[nxt] = time.perf_counter()
                if not dp.prefetch(base + offs[nb], blens[nb]):
                    break
                pre.add(nxt)
                nxt += 1
            return t, s

        if args.loop == "poll":
            # the host never blocks on one thing while another is due: a parity frees ->
            # submit the next step at once (its ingest overlaps the routing half in flight);
            # an egress lands -> its deliveries are stamped when it does
            from collections import deque
            pq, dq = deque(), deque()
            issued = 0
            last = time.perf_counter()
            while issued < n or pq or dq:
                prog = False
                if issued < n and len(pq) < 2:
                    pq.append(submit_next())
                    issued += 1
                    prog = True
                    if measure:
                        now = time.perf_counter()
                        phases.append([round((now - last) * 1e3, 4)])
                        last = now
                if pq and dp.step_done(pq[0][0]):
                    t, s = pq.popleft()
                    account(dp.finish(t, collect=False, wait_egress=False), s)
                    dq.append((t, s))
                    prog = True
                while dq and dp.egress_done(dq[0][0]):
                    t, s = dq.popleft()
                    ready(s)
                    prog = True
                if not prog and issued == n and not pq:   # draining: block on the last egress
                    t, s = dq.popleft()
                    dp.egress_wait(t)
                    ready(s)
            return dl, pb, hist, eg

        for i in range(n):
            tp = [time.perf_counter()]   # host time per phase of this iteration (slowest kept)
            b = step_i % args.blocks
            if step_i not in pre:   # (a prefetched step's clock started when its bytes were queued)
                sub_t[step_i] = time.perf_counter()
            pre.discard(step_i)
            if storm:   # ack-all each step, nack-all-requeue every 4th: a redelivery storm
                cs = extra["nack" if step_i % 4 == 3 else "ack"][b]
                if flow["paused"]:
                    flow["paused_steps"] += 1
                    sg = cs
                else:
                    sg = np.concatenate([segs[b], cs])
                pending.append((submit(sg, base + offs[b], blens[b]), step_i))
            else:
                pending.append((submit(segs[b], base + offs[b], blens[b]), step_i))
            tp.append(time.perf_counter())
            step_i += 1
            # the next steps of this run whose bytes are not queued yet (in order: the engine
            # queues each call's payload for the next such step)
            nxt = max(step_i, max(pre) + 1 if pre else step_i)
            while args.prefetch and nxt < min(step_i + args.prefetch, end):
                nb = nxt % args.blocks
                sub_t[nxt] = time.perf_counter()
                if not dp.prefetch(base + offs[nb], blens[nb]):
                    break
                pre.add(nxt)
                nxt += 1
            tp.append(time.perf_counter())
            # step i-2, waited on at the end of the previous iteration: collected only now,
            # behind step i's submit (its bookkeeping is off the wait -> next-H2D path); then
            # its egress (the D2H its last kernel started a step ago: in host memory by now)
            if waited:
                t2, s2 = waited.pop()
                account(dp.finish(t2, collect=False, wait_egress=False, waited=True), s2)
                done.append((t2, s2))
            while done:
                t2, s2 = done.pop(0)
                dp.egress_wait(t2)
                ready(s2)
            tp.append(time.perf_counter())
            # step i-1's kernels (the host's only per-step wait on them): frees its parity, so
            # the next iteration's submit -- step i+1's ingress H2D -- follows the wait at once
            if len(pending) > npar - 1:
                t, s = pending.pop(0)
                dp.wait(t)
                waited.append((t, s))
                # the next step's payload H2D right behind the wait (its parity is free now):
                # the copy engine restarts without waiting for the loop's bookkeeping and
                # submit; the step's latency clock starts here, where its bytes are queued
                if args.h2d_at_wait and not args.prefetch and not storm and world == 1 and step_i < end \
                        and step_i not in pre:
                    nb = step_i % args.blocks
                    sub_t[step_i] = time.perf_counter()
                    if dp.prefetch(base + offs[nb], blens[nb]):
                        pre.add(step_i)
            tp.append(time.perf_counter())
            if measure:
                ph = [round((b2 - a2) * 1e3, 3) for a2, b2 in zip(tp, tp[1:])]
                phases.append(ph)
                if sum(ph) > slow["ms"]:
                    slow.update(ms=round(sum(ph), 3), step=i, phases_ms=ph)
        for t, s in waited:
            account(dp.finish(t, collect=False, wait_egress=False, waited=True), s)
            done.append((t, s))
        for t, s in done:
            dp.egress_wait(t)
            ready(s)
        for t, s in pending:
            account(dp.finish(t, collect=False, wait_egress=True), s)
            ready(s)
        return dl, pb, hist, eg

    # the host loop is the pipeline's driver: no collector pause inside the window.  Collected
    # before the warm-up steps, which then re-warm the allocator (a collection right before
    # the window made the first timed submit 0.6 ms slower, round 5: profiles/r5_summary.md)
    import gc
    gc.collect()
    gc.disable()
    run(args.warmup)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    dp.eng.sync()
    if shards > 1 and not native:
        dp.exchanger.bytes_sent = 0
    dp.eng.host_times(True)
    t0 = time.perf_counter()
    dl, pb, hist, eg = run(args.steps, measure=True)
    dp.eng.sync()
    torch.cuda.synchronize()
    gc.enable()
    if dist:
        dist.barrier()
    t = time.perf_counter() - t0
    n_ref_timed, wire_timed = nref[0], wire[0]
    verified = None
    if args.egress_ref:   # two more steps, each finished and checked on its own (every rank)
        verified = 0
        for _ in range(2):
            b = step_i % args.blocks
            tk = submit(segs[b], base + offs[b], blens[b])
            step_i += 1
            dp.finish(tk, collect=False, wait_egress=True)
            verified += verify_egress(dp, base, sum(blens) + 64, [tk])
    c = dp.eng.counters((step_i - 1) % npar)
    errs = {k: c[k] for k in ("n_dropped_nomem", "n_ring_full", "n_unknown_exchange", "n_unroutable",
                              "n_routed_msgs", "n_pairs", "n_deliv", "n_live_msgs") if c[k]}

    vals = np.array([t, dl, pb, eg], np.float64)
    if dist:
        rdev = "cuda" if backend == "nccl" else "cpu"
        tt = torch.tensor([t], dtype=torch.float64, device=rdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        ss = torch.tensor(vals[1:], dtype=torch.float64, device=rdev)
        dist.all_reduce(ss, op=dist.ReduceOp.SUM)
        hh = torch.tensor(hist, dtype=torch.float64, device=rdev)
        dist.all_reduce(hh, op=dist.ReduceOp.SUM)
        t = float(tt.item())
        dl, pb, eg = (float(x) for x in ss.tolist())
        hist = hh.cpu().numpy()
    ms_step = 1000.0 * t / args.steps
    # p50 publish->deliver, measured on the host clock per delivery: from the submit of the
    # step that carried the publish to the moment the delivering step's egress bytes were in
    # host memory (the step pipeline, queueing and the D2H included; no TCP)
    lat = np.array(lat_w, np.float64).reshape(-1, 2)
    p50_ms = p99_ms = None
    if len(lat):
        order = np.argsort(lat[:, 0])
        cw = np.cumsum(lat[order, 1])
        p50_ms = 1000.0 * float(lat[order[np.searchsorted(cw, 0.5 * cw[-1])], 0])
        p99_ms = 1000.0 * float(lat[order[min(len(order) - 1, np.searchsorted(cw, 0.99 * cw[-1]))], 0])
    if dist:   # the slowest rank's median
        lt = torch.tensor([p50_ms or 0.0, p99_ms or 0.0], dtype=torch.float64, device=rdev)
        dist.all_reduce(lt, op=dist.ReduceOp.MAX)
        p50_ms, p99_ms = (float(x) for x in lt.tolist())
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": dl / t,
            "unit": "msgs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "uint8 (AMQP wire bytes; no floating-point compute)",
            "data": "synthetic AMQP 0-9-1 publish traffic (random 1 KB bodies), empty-init broker state",
            "config": {
                "model": (f"BASELINE config 3: fanout exchange -> {qtot} queues ({Q} per GPU), {args.body} B msgs, "
                          "auto-ack, non-persistent; value = deliveries/s") if fan else
                         (f"BASELINE config 5: direct exchange, {P} producers x {Q} manual-ack consumers per GPU "
                          f"(prefetch 512), ack-all each step, nack-all-requeue every 4th step, producer flow "
                          f"pause above 1 GiB; value = deliveries/s incl. redeliveries") if storm else
                         (f"BASELINE config 2: 1 topic exchange, {Q} bound queues per GPU, {args.body} B msgs, "
                          "auto-ack, non-persistent"),
                "global_batch": int(round(mps * world)),
                "seq_len": args.body,
                "parallelism": (f"queue-sharded x{world}: one broker, cross-GPU routing by "
                                + (("engine-native grouped RCCL send/recv over xGMI, counts via host shared memory"
                                    if backend == "nccl" else
                                    "engine-native RCCL code path through the TEST STAND-IN library (one-GPU "
                                    "rehearsal: shared memory + hipMemcpy, not xGMI; no scaling number)"
                                    if dp.info.get("rccl_standin") else
                                    "engine-native shared-memory exchange (host-staged)")
                                   if native else
                                   "RCCL all-to-all" if backend == "nccl" else f"{backend} all-to-all staged through the host")
                                + (" (pipelined, +1 step for cross-GPU messages)" if args.exchange_lag else "")
                                if shards > 1 else
                                (f"x{world} independent broker shards" if world > 1 else "single GPU")),
                "producers_per_gpu": P,
                "consumers_per_gpu": Q,
                "bytes_per_msg_on_wire": msg_bytes,
            },
            "p50_latency_ms": p50_ms,
            "p99_latency_ms": p99_ms,
            "published_msgs_per_s": pb / t,
            "egress_GBps": eg / t / 1e9,
            "d2h_bytes_per_step": eg / max(1, args.steps * world),
            "wire_bytes_per_step": wire_timed / max(1, args.steps),
            "egress_ref": ({"referenced_deliveries": n_ref_timed, "verified": verified,
                            "note": "bodies of deliveries referenced in the ingress pool block of their own step "
                                    "(never rewritten; resubmitted 8 steps later); the D2H carries frames + "
                                    "gather table"} if args.egress_ref else None),
            "latency_note": "measured per delivery on the host clock: submit of the publishing step -> egress "
                            "bytes of the delivering step in host memory (no TCP; bench/gpu_server_e2e.py "
                            "measures client-to-client over TCP)",
            "diag": errs,
            "slowest_iteration": slow,
            "first_iterations_ms": phases[:3],
            "iteration_phases_ms_median": ([round(float(np.median([p[k] for p in phases if len(p) > k])), 4)
                                            for k in range(max(len(p) for p in phases))] if phases else None),
            "host_us_per_step": {k: round(v * 1e6 / args.steps, 1) for k, v in dp.eng.host_times(False).items()},
            "egress": dp.eng.egress_stats(),
            "storm": ({"requeued_msgs": flow["requeued"], "flow_paused_steps": flow["paused_steps"]}
                      if storm else None),
            "cross_gpu_bytes_per_s": (dp.exchanger.bytes_sent * world / t) if shards > 1 and not native else None,
            "exchange": ((args.xchg + " (" + (os.environ.get("CHANAMQ_BENCH_XCHG") or ("rccl" if backend == "nccl" else "shm"))
                          + (", librccl stand-in" if os.environ.get("CHANAMQ_RCCL_LIB") else "") + ")") if native else args.xchg)
                         if shards > 1 else None,
            "async_exchange": bool(args.async_x) if shards > 1 else None,
            "prefetch": bool(args.prefetch), "parities": npar, "h2d_alt": bool(args.h2d_alt), "h2d_hsa": bool(args.h2d_hsa), "h2d_at_wait": bool(args.h2d_at_wait),
            "chunk_bytes_per_producer": args.chunk,
            "post_soak_s": args.soak_s,
        }
        print(json.dumps(out), flush=True)
    if args.soak_s > 0:
        # untimed: the same step count on every rank (ms_step is the max over ranks), so the
        # lockstep exchange stays matched
        run(max(1, min(20000, int(args.soak_s * 1000.0 / max(ms_step, 1e-3)))))
        dp.eng.sync()
        torch.cuda.synchronize()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
