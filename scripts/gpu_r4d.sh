#!/bin/bash
# Round 4 (d): the full GPU suite (unpauses now ride the next step), the driver's bench
# line, config 2 with Basic.Get pollers (lock-free Get path) and config 4 (body log).
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4d}
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail 8 --timeout 400 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest_gpu.log; tail -12 $O/pytest_gpu.log | grep -E "passed|failed|FAILED|ERROR"; fatal $rc pytest
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -2 $O/smoke.log; fatal $rc smoke
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err; rc=$?; fatal $rc bench
grep -o '"value": [0-9.e+]*\|"p50_latency_ms": [0-9.]*' $O/bench_default.json | tr '\n' ' '; echo
timeout -k 10 400 python -u bench/gpu_server_e2e.py --seconds 4 --io-threads 8 --only config2 --paced 0 --getters 4 \
  --out $O/e2e_config2_getters.json > $O/e2e_config2_getters.log 2>&1
rc=$?; fatal $rc e2e; cut -c1-420 $O/e2e_config2_getters.log | grep "^{" | tail -3
timeout -k 10 300 python -u bench/gpu_server_e2e.py --seconds 4 --io-threads 8 --only config4 --paced 0.5 \
  --out $O/e2e_config4.json > $O/e2e_config4.log 2>&1
rc=$?; fatal $rc e2e4; cut -c1-420 $O/e2e_config4.log | grep "^{" | tail -3
exit 0
