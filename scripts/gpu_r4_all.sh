#!/bin/bash
# Round 4, one box for everything: the full GPU suite (no -x: every test reports), the
# headline bench at several step sizes, a kernel trace of the overlapped step, the native
# exchange checks, and config 2 over TCP with Basic.Get pollers + paced (tail stages).
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4_all}
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail 8 --timeout 400 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest_gpu.log; tail -12 $O/pytest_gpu.log | grep -E "passed|failed|FAILED|ERROR"; fatal $rc pytest
for ch in ${CHUNKS:-65536 32768 24576}; do
  for k in 20 200; do
    timeout -k 10 120 python bench.py --steps $k --warmup 5 --soak-s 0 --chunk $ch > $O/bench_c${ch}_k$k.json 2> $O/bench_c${ch}_k$k.err
    rc=$?; fatal $rc bench; [ $rc -ne 0 ] && { tail -5 $O/bench_c${ch}_k$k.err; continue; }
    python -c "import json,sys; d=json.load(open('$O/bench_c${ch}_k$k.json')); print($ch, $k, round(d['value']/1e6,2), 'M', round(d['p50_latency_ms'],3), round(d['p99_latency_ms'],3), round(d['ms_per_step'],3))"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- python3 bench.py --steps 40 --warmup 5 --soak-s 0 --chunk 32768 > $O/trace.log 2>&1
rc=$?; fatal $rc trace
if [ $rc -eq 0 ]; then python3 scripts/step_gaps.py $O/t > $O/gaps_c32768.csv; tail -4 $O/gaps_c32768.csv; python3 scripts/overlap_timeline.py $O/t > $O/overlap_c32768.txt 2>&1; tail -6 $O/overlap_c32768.txt; fi
rm -rf $O/t
RUN=$(basename $O)_xchg bash scripts/gpu_r4_xchg.sh; fatal $? xchg
timeout -k 10 400 python -u bench/gpu_server_e2e.py --seconds 4 --io-threads 8 --only config2 --paced 0.5 --getters 4 \
  --out $O/e2e_config2.json > $O/e2e_config2.log 2>&1
rc=$?; fatal $rc e2e; grep -v "^{" $O/e2e_config2.log | tail -3; cut -c1-400 $O/e2e_config2.log | grep "^{" | tail -3
exit 0
