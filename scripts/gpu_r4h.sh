#!/bin/bash
# Round 4 (h): payload prefetch 1 vs 2 steps ahead (own H2D stream), the K=20 window; the
# engine/broker GPU tests (the pipelined front end prefetches too).
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4h}
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
summ() { python -c "
import json,sys; s=open('$1').read(); d=json.loads(s[s.index('{'):])
print('$2', round(d['value']/1e6,2), 'M p50', round(d['p50_latency_ms'],3), 'p99', round(d['p99_latency_ms'],3), 'ms/step', round(d['ms_per_step'],3), d['host_us_per_step'])"; }
for cfg in ${BENCH:-"32768 20 1" "32768 20 2" "40960 20 2" "49152 20 1" "49152 20 2" "65536 20 1" "65536 20 2" "32768 200 2" "65536 200 2"}; do
  set -- $cfg
  f=$O/bench_c$1_k$2_p$3
  timeout -k 10 120 python bench.py --steps $2 --warmup 5 --soak-s 0 --chunk $1 --prefetch $3 > $f.json 2> $f.err
  rc=$?; fatal $rc bench; [ $rc -ne 0 ] && { tail -5 $f.err; continue; }
  summ $f.json "chunk $1 K=$2 prefetch $3"
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_dataplane.py tests/test_gpu_broker.py -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest.log; tail -3 $O/pytest.log | grep -E "passed|failed"; fatal $rc pytest
exit 0
