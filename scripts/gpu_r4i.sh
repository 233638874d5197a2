#!/bin/bash
# Round 4 (i): egress copy queued behind the step on the GPU (kernel copy, sized on the
# device) vs the host-issued SDMA copy, at the driver's K=20 / W=5.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4i}
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
summ() { python -c "
import json,sys; s=open('$1').read(); d=json.loads(s[s.index('{'):])
print('$2', round(d['value']/1e6,2), 'M p50', round(d['p50_latency_ms'],3), 'p99', round(d['p99_latency_ms'],3), 'ms/step', round(d['ms_per_step'],3), d['host_us_per_step'])"; }
for cfg in ${BENCH:-"32768 sdma 16" "32768 kernel 16" "32768 kernel 32" "49152 kernel 32" "65536 kernel 32" "65536 sdma 16"}; do
  set -- $cfg
  f=$O/bench_c$1_$2_w$3
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --soak-s 0 --chunk $1 --prefetch ${PRE:-2} --copy-engine $2 --copy-wgs $3 > $f.json 2> $f.err
  rc=$?; fatal $rc bench; [ $rc -ne 0 ] && { tail -5 $f.err; continue; }
  summ $f.json "chunk $1 $2 wgs $3"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_dataplane.py -x -q --timeout 400 --timeout-method thread -p no:cacheprovider -k "copykernel or graph" > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest.log; tail -3 $O/pytest.log | grep -E "passed|failed"; fatal $rc pytest
timeout -k 10 300 python -u bench/gpu_server_e2e.py --io-threads 8 --wal-soak 30 --out $O/e2e_config4_soak30.json > $O/e2e_config4_soak.log 2>&1
rc=$?; fatal $rc soak; grep "^{" $O/e2e_config4_soak.log | cut -c1-600 | tail -1
exit 0
