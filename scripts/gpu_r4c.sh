#!/bin/bash
# Round 4 (c): egress D2H over one vs two SDMA engines at the headline step sizes, plus the
# Basic.Get pollers next to config 2 (separate process now).
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4c}
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
summ() { python -c "
import json,sys; s=open('$1').read(); d=json.loads(s[s.index('{'):])
print('$2', round(d['value']/1e6,2), 'M p50', round(d['p50_latency_ms'],3), 'p99', round(d['p99_latency_ms'],3), 'ms/step', round(d['ms_per_step'],3), d['host_us_per_step'])"; }
for cfg in ${BENCH:-"32768 200 1" "32768 200 2" "65536 200 1" "65536 200 2" "32768 20 2" "49152 20 2" "65536 20 2" "40960 20 2"}; do
  set -- $cfg
  f=$O/bench_c$1_k$2_s$3
  timeout -k 10 120 python bench.py --steps $2 --warmup 5 --soak-s 0 --chunk $1 --sdma-split $3 > $f.json 2> $f.err
  rc=$?; fatal $rc bench; [ $rc -ne 0 ] && { tail -5 $f.err; continue; }
  summ $f.json "chunk $1 K=$2 split $3"
done
timeout -k 10 400 python -u bench/gpu_server_e2e.py --seconds 4 --io-threads 8 --only config2 --paced 0 --getters 4 \
  --out $O/e2e_config2_getters.json > $O/e2e_config2_getters.log 2>&1
rc=$?; fatal $rc e2e; cut -c1-500 $O/e2e_config2_getters.log | grep "^{" | tail -3
exit 0
