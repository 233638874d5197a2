#!/bin/bash
# Round 4 (b): the full GPU suite, the headline bench with / without the early ingress H2D
# (prefetch) over step sizes, a kernel + memory-copy trace of the overlapped pipeline, and
# configs 4 (store) and 2 (paced tail) over TCP.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4b}
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
if [ -z "$SKIP_SUITE" ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail 8 --timeout 400 --timeout-method thread -p no:cacheprovider ${SUITE:-} > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest_gpu.log; tail -12 $O/pytest_gpu.log | grep -E "passed|failed|FAILED|ERROR"; fatal $rc pytest
fi
summ() { python -c "
import json,sys; s=open('$1').read(); d=json.loads(s[s.index('{'):])
print('$2', round(d['value']/1e6,2), 'M p50', round(d['p50_latency_ms'],3), 'p99', round(d['p99_latency_ms'],3), 'ms/step', round(d['ms_per_step'],3), d['host_us_per_step'])"; }
for cfg in ${BENCH:-"65536 20 1" "65536 20 0" "49152 20 1" "32768 20 1" "32768 20 0" "24576 20 1" "16384 20 1" "65536 200 1" "32768 200 1" "24576 200 1"}; do
  set -- $cfg
  f=$O/bench_c$1_k$2_p$3
  timeout -k 10 120 python bench.py --steps $2 --warmup 5 --soak-s 0 --chunk $1 --prefetch $3 > $f.json 2> $f.err
  rc=$?; fatal $rc bench; [ $rc -ne 0 ] && { tail -5 $f.err; continue; }
  summ $f.json "chunk $1 K=$2 prefetch $3"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/t -o run -- python3 bench.py --steps 40 --warmup 5 --soak-s 0 --chunk 32768 --prefetch 1 > $O/trace.log 2>&1
rc=$?; fatal $rc trace
if [ $rc -eq 0 ]; then
  python3 scripts/step_gaps.py $O/t > $O/gaps_c32768.csv; tail -4 $O/gaps_c32768.csv
  python3 scripts/overlap_timeline.py $O/t > $O/overlap_c32768.txt 2>&1; tail -6 $O/overlap_c32768.txt
  mkdir -p $O/trace_csv
  for f in $(find $O/t -name "*.csv"); do gzip -c "$f" > $O/trace_csv/$(basename "$f").gz; done
fi
rm -rf $O/t
timeout -k 10 300 python -u bench/gpu_server_e2e.py --seconds 4 --io-threads 8 --only config4 --paced 0 \
  --out $O/e2e_config4.json > $O/e2e_config4.log 2>&1
rc=$?; fatal $rc e2e4; cut -c1-700 $O/e2e_config4.log | grep "^{" | tail -2
timeout -k 10 300 python -u bench/gpu_server_e2e.py --seconds 4 --io-threads 8 --only config2 --paced 0.5 \
  --out $O/e2e_config2.json > $O/e2e_config2.log 2>&1
rc=$?; fatal $rc e2e2; cut -c1-400 $O/e2e_config2.log | grep "^{" | tail -3
exit 0
