#!/bin/bash
# One parameterised driver for every GPU-box run of this repo (replaces the per-round
# one-off scripts).  Usage, from the repo root on the box (gpurun -- bash scripts/gpu.sh ...):
#
#   bash scripts/gpu.sh TASK [TASK ...]
#
# Tasks run in order; the first task that fails or trips a fatal status (time limit, abort,
# segfault) ends the run -- nothing else touches the GPU after it.  Output: gpurun_out/$RUN/
# (RUN defaults to "gpu").
#
#   suite       pytest -m gpu -x (as the driver runs it), one process
#   suite_all   pytest -m gpu without -x (every test reports; stops after 8 failures)
#   smoke       __graft_entry__.smoke()
#   bench       bench.py at the driver's K=20 / W=5, once per CHUNKS entry (default: the
#               bench's default step), REPEAT times each (default 1)
#   bench200    the same at K=200 (steady state)
#   sweep       bench.py once per SWEEP entry ("label=--args;label=--args"), REPEAT times, K=${K:-20}
#   trace       rocprofv3 kernel + memory-copy trace of bench.py (CHUNK, default 32768),
#               then the step timeline / overlap / gap summaries
#   stats       rocprofv3 --kernel-trace --stats of bench.py (per-kernel time table)
#   pmc         hardware counters per kernel of the headline step, one rocprofv3 --pmc pass
#               per counter group (PMC_GROUPS overrides), each under its own time limit
#   xchg        the single-rank RCCL exchange test, then the 2- and 4-rank native / torch
#               exchange rehearsal on this one GPU (gloo launcher => shared-memory backend)
#   xchg8       the 8-rank shared-memory rehearsal on this one GPU (asynchronous and synchronous
#               exchange; the stepper's exchange wait per step is host_us_per_step.exchange)
#   e2e         bench/gpu_server_e2e.py, every spec, paced at 50 % (E2E_ARGS appended; IOT io
#               threads, LG load-generator threads, TAG output-name suffix)
#   e2e_c2      config 2 only over TCP, paced at 50 % (E2E_ARGS appended)
#   churn       config 2 paced at 50 % next to connection / consumer churn (E2E_ARGS appended)
#   cold        bench/cold_paging.py: a backlog through all three body tiers, drained under live
#               traffic (COLD_ARGS appended)
#   sharded     the sharded-server GPU tests
#   sharded_e2e config 2 on the 2-rank sharded server over TCP, local vs remote consumers
#   tests:PAT   pytest -m gpu -x -k PAT ('+' = or)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${RUN:-gpu}
mkdir -p "$O"
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit "$1";; esac; }
ok() { local rc=$1; fatal "$rc" "$2"; [ "$rc" -ne 0 ] && { echo "$2 failed (exit $rc)"; exit "$rc"; }; return 0; }
line() {   # one bench JSON line -> a short summary
  python3 - "$1" <<'EOF'
import json, sys
s = open(sys.argv[1]).read()
d = json.loads(s[s.index("{"):].splitlines()[0])
print(sys.argv[1].split("/")[-1], round(d["value"] / 1e6, 2), "M msgs/s  p50", round(d["p50_latency_ms"] or 0, 3),
      "p99", round(d["p99_latency_ms"] or 0, 3), "ms/step", round(d["ms_per_step"], 3), "host", d.get("host_us_per_step"))
EOF
}
PYT="python -u -m pytest -p no:cacheprovider --timeout 400 --timeout-method thread"

for T in "$@"; do
  case $T in
  suite)
    timeout -k 10 1000 $PYT tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
    rc=$?; echo "pytest exit $rc" >> $O/pytest_gpu.log; tail -4 $O/pytest_gpu.log; ok $rc suite ;;
  suite_all)
    timeout -k 10 1100 $PYT tests -m gpu -v --maxfail 8 > $O/pytest_gpu_all.log 2>&1
    rc=$?; echo "pytest exit $rc" >> $O/pytest_gpu_all.log
    grep -E "FAILED|ERROR" $O/pytest_gpu_all.log | head -20; tail -2 $O/pytest_gpu_all.log; ok $rc suite_all ;;
  smoke)
    timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
    rc=$?; tail -1 $O/smoke.log; ok $rc smoke ;;
  bench|bench200)
    K=20; [ "$T" = bench200 ] && K=200
    for ch in ${CHUNKS:-default}; do
      for r in $(seq 1 "${REPEAT:-1}"); do
        f=$O/${T}_c${ch}_r$r.json
        CA=""; [ "$ch" != default ] && CA="--chunk $ch"
        timeout -k 10 150 python bench.py --gpus 1 --steps $K --warmup 5 --soak-s 0 $CA $BENCH_ARGS > $f 2> ${f%.json}.err
        ok $? bench; line $f
      done
    done ;;
  sweep)   # SWEEP="label1=--args ...;label2=--args ..." -> bench.py K=${K:-20} once per entry, REPEAT times
    IFS=';' read -ra ENTRIES <<< "$SWEEP"
    for ent in "${ENTRIES[@]}"; do
      lab=${ent%%=*}; args=${ent#*=}
      for r in $(seq 1 "${REPEAT:-1}"); do
        f=$O/sweep_${lab}_r$r.json
        timeout -k 10 150 python bench.py --gpus 1 --steps ${K:-20} --warmup 5 --soak-s 0 $args > $f 2> ${f%.json}.err
        ok $? "sweep $lab"; line $f
      done
    done ;;
  trace)
    ch=${CHUNK:-32768}
    timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/t -o run -- \
      python3 bench.py --steps 40 --warmup 5 --soak-s 0 --chunk $ch $BENCH_ARGS > $O/trace.log 2>&1
    ok $? trace
    python3 scripts/pipeline_timeline.py $O/t > $O/timeline_c$ch.txt 2>&1; cat $O/timeline_c$ch.txt
    python3 scripts/overlap_timeline.py $O/t > $O/overlap_c$ch.txt 2>&1; tail -4 $O/overlap_c$ch.txt
    python3 scripts/step_gaps.py $O/t > $O/gaps_c$ch.csv 2>&1; tail -4 $O/gaps_c$ch.csv
    mkdir -p $O/trace_c$ch
    for f in $(find $O/t -name "*kernel_trace.csv" -o -name "*memory_copy_trace.csv"); do gzip -c $f > $O/trace_c$ch/$(basename $f).gz; done
    rm -rf $O/t ;;
  trace_host)   # the trace above plus the host's roctx ranges (submit / prefetch / waits)
    ch=${CHUNK:-32768}
    timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --output-format csv -d $O/th -o run -- \
      python3 bench.py --steps 40 --warmup 5 --soak-s 0 --chunk $ch $BENCH_ARGS > $O/trace_host.log 2>&1
    ok $? trace_host
    mkdir -p $O/trace_host_c$ch
    for f in $(find $O/th -name "*kernel_trace.csv" -o -name "*memory_copy_trace.csv" -o -name "*marker_api_trace.csv"); do gzip -c $f > $O/trace_host_c$ch/$(basename $f).gz; done
    rm -rf $O/th ;;
  stats)
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s -o run -- \
      python3 bench.py --steps 20 --warmup 5 --soak-s 0 $BENCH_ARGS > $O/stats.log 2>&1
    ok $? stats
    f=$(find $O/s -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" $O/kernel_stats.csv && head -30 $O/kernel_stats.csv
    rm -rf $O/s ;;
  pmc)
    k=0
    GROUPS_=${PMC_GROUPS:-"SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_VMEM_RD,SQ_INSTS_LDS;SQ_INSTS_VALU_MFMA_MOPS_I8,SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_MFMA,SQ_LDS_BANK_CONFLICT,SQ_INSTS_VMEM_WR,SQ_ACTIVE_INST_ANY;FETCH_SIZE;WRITE_SIZE"}
    IFS=';' read -ra GS <<< "$GROUPS_"
    for G in "${GS[@]}"; do
      k=$((k+1))
      timeout -s KILL 90 rocprofv3 --pmc ${G//,/ } --output-format csv -d $O/p$k -o run -- \
        python3 bench.py --steps 6 --warmup 2 --soak-s 0 $BENCH_ARGS > $O/pmc_p$k.log 2>&1
      ok $? "pmc group $k"
      python3 scripts/pmc_summary.py $O/p$k > $O/pmc$k.csv && cat $O/pmc$k.csv
      rm -rf $O/p$k
    done ;;
  xchg)
    timeout -k 10 200 $PYT tests/test_gpu_sharded.py -m gpu -x -v -k rccl_single > $O/pytest_rccl.log 2>&1
    rc=$?; tail -3 $O/pytest_rccl.log; ok $rc rccl_single
    for n in 2 4; do
      for x in native torch; do
        f=$O/bench_${n}r_$x${TAG:-}.json
        CHANAMQ_BENCH_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
          --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 30 --warmup 5 --soak-s 0 \
          --xchg $x $BENCH_ARGS > $f 2> ${f%.json}.err
        ok $? "xchg ${n}r $x"; line $f
      done
    done ;;
  xchg_rccl)   # bench.py's RCCL exchange (RcclXchg) at 2 / 4 / 8 ranks on this one GPU through the tests'
               # librccl stand-in (real RCCL refuses several ranks on one device): a rehearsal, not scaling
    SO=$(python3 -c "from chanamq_amd import ops; print(ops.build_rccl_standin())") || { echo "no stand-in"; exit 1; }
    for n in ${RANKS:-2 4 8}; do
      for ax in ${ASYNC:-0 1}; do
        f=$O/bench_${n}r_rccl_async$ax${TAG:-}.json
        CHANAMQ_BENCH_BACKEND=gloo CHANAMQ_BENCH_XCHG=rccl CHANAMQ_RCCL_LIB=$SO CHANAMQ_RCCL_STANDIN_OK=1 \
          timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
          --master-addr 127.0.0.1 --master-port $((29620 + n + 10 * ax)) bench.py --gpus $n --steps 30 --warmup 5 \
          --soak-s 0 --xchg native --async-x $ax $XCHG8_ARGS > $f 2> ${f%.json}.err
        ok $? "xchg_rccl ${n}r async $ax"; line $f
      done
    done ;;
  xchg8)   # the 8-rank shared-memory rehearsal on this one GPU, asynchronous exchange then synchronous
    for ax in 1 0; do
      f=$O/bench_8r_shm_async$ax${TAG:-}.json
      CHANAMQ_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
        --master-addr 127.0.0.1 --master-port $((29610 + ax)) bench.py --gpus 8 --steps 30 --warmup 5 --soak-s 0 \
        --xchg native --async-x $ax $XCHG8_ARGS > $f 2> ${f%.json}.err
      ok $? "xchg8 async $ax"; line $f
    done ;;
  e2e)
    timeout -k 10 900 python -u bench/gpu_server_e2e.py --seconds 4 --io-threads ${IOT:-8} --paced 0.5 \
      --loadgen-threads ${LG:-12} --out $O/e2e_all_specs${TAG:-}.json $E2E_ARGS > $O/e2e${TAG:-}.log 2>&1
    rc=$?; tail -12 $O/e2e${TAG:-}.log | cut -c1-600; ok $rc e2e ;;
  e2e_c2)
    timeout -k 10 400 python -u bench/gpu_server_e2e.py --seconds 4 --io-threads ${IOT:-8} --only config2 --paced 0.5 \
      --loadgen-threads ${LG:-12} --out $O/e2e_c2${TAG:-}.json $E2E_ARGS > $O/e2e_c2${TAG:-}.log 2>&1
    rc=$?; tail -4 $O/e2e_c2${TAG:-}.log | cut -c1-600; ok $rc e2e_c2 ;;
  churn)
    timeout -k 10 400 python -u bench/gpu_server_e2e.py --seconds 5 --io-threads ${IOT:-8} --only config2 --paced 0.5 \
      --churn --out $O/e2e_churn.json $E2E_ARGS > $O/e2e_churn.log 2>&1
    rc=$?; tail -4 $O/e2e_churn.log | cut -c1-800; ok $rc churn ;;
  cold)   # timed cold paging: backlog through HBM log -> host ring -> disk, drained under live traffic
    timeout -k 10 300 python -u bench/cold_paging.py --out $O/cold_paging.json $COLD_ARGS > $O/cold_paging.log 2>&1
    rc=$?; tail -3 $O/cold_paging.log | cut -c1-600; ok $rc cold ;;
  sharded_e2e)   # config 2 on the 2-rank sharded server, consumers on the owner rank vs remote
    timeout -k 10 600 python -u bench/gpu_server_e2e.py --sharded 2 --only config2 --seconds 4 --io-threads 2 \
      --out $O/sharded2_config2_local_remote${TAG:-}.json $E2E_ARGS > $O/sharded_e2e${TAG:-}.log 2>&1
    rc=$?; tail -6 $O/sharded_e2e${TAG:-}.log | cut -c1-400; ok $rc sharded_e2e ;;
  sharded)
    timeout -k 10 700 $PYT tests/test_gpu_sharded.py tests/test_gpu_sharded_server.py -m gpu -x -v > $O/pytest_sharded.log 2>&1
    rc=$?; tail -4 $O/pytest_sharded.log; ok $rc sharded ;;
  tests:*)   # PAT: a -k expression, '+' between alternatives (tests:dataplane+scale = -k "dataplane or scale")
    K_EXPR=${T#tests:}; K_EXPR=${K_EXPR//+/ or }
    timeout -k 10 900 $PYT tests -m gpu -x -v -k "$K_EXPR" > $O/pytest_k.log 2>&1
    rc=$?; grep -E "PASSED|FAILED|ERROR" $O/pytest_k.log | tail -30; tail -2 $O/pytest_k.log; ok $rc "tests ${T#tests:}" ;;
  *) echo "unknown task $T"; exit 2 ;;
  esac
done
exit 0
