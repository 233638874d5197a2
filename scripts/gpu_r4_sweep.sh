#!/bin/bash
# Round 4: step-size sweep of the headline bench (bytes per producer per step), the new
# record-budget test, K=20/W=5 like the driver and K=200 for a steadier number.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4_sweep}
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_broker.py -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "record_budget or purge_of_more" > $O/pytest_budget.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest_budget.log; tail -3 $O/pytest_budget.log; [ $rc -ne 0 ] && exit $rc
for ch in ${CHUNKS:-65536 32768 16384 8192 4096}; do
  for k in 20 200; do
    timeout -k 10 120 python bench.py --steps $k --warmup 5 --soak-s 0 --chunk $ch $EXTRA > $O/bench_c${ch}_k$k.json 2> $O/bench_c${ch}_k$k.err
    rc=$?; [ $rc -ne 0 ] && { tail -5 $O/bench_c${ch}_k$k.err; exit $rc; }
    python -c "import json,sys; d=json.load(open('$O/bench_c${ch}_k$k.json')); print($ch, $k, round(d['value']/1e6,2), 'M', round(d['p50_latency_ms'],3), round(d['p99_latency_ms'],3), round(d['ms_per_step'],3), d['host_us_per_step'])"
  done
done
