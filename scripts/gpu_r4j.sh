#!/bin/bash
# Round 4 (j): prefetch depth and the GPU-queued egress copy at the driver's K=20 / W=5,
# the engine + broker GPU tests, and a 30 s config-4 soak with reopen / recovery times.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4j}
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
summ() { python -c "
import json,sys; s=open('$1').read(); d=json.loads(s[s.index('{'):])
print('$2', round(d['value']/1e6,2), 'M p50', round(d['p50_latency_ms'],3), 'p99', round(d['p99_latency_ms'],3), 'ms/step', round(d['ms_per_step'],3), d['host_us_per_step'])"; }
for cfg in ${BENCH:-"32768 1 sdma 16" "32768 2 sdma 16" "32768 2 kernel 32" "49152 2 sdma 16" "49152 2 kernel 32" "65536 1 sdma 16" "65536 2 sdma 16" "65536 2 kernel 32" "24576 2 kernel 32"}; do
  set -- $cfg
  f=$O/bench_c$1_p$2_$3$4
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --soak-s 0 --chunk $1 --prefetch $2 --copy-engine $3 --copy-wgs $4 > $f.json 2> $f.err
  rc=$?; fatal $rc bench; [ $rc -ne 0 ] && { tail -5 $f.err; continue; }
  summ $f.json "chunk $1 prefetch $2 $3 wgs $4"
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_dataplane.py tests/test_gpu_broker.py -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest.log; tail -3 $O/pytest.log | grep -E "passed|failed"; fatal $rc pytest
timeout -k 10 300 python -u bench/gpu_server_e2e.py --io-threads 8 --wal-soak 30 --out $O/e2e_config4_soak30.json > $O/e2e_config4_soak.log 2>&1
rc=$?; fatal $rc soak; grep "^{" $O/e2e_config4_soak.log | cut -c1-700 | tail -1
exit 0
