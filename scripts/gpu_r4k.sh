#!/bin/bash
# Round 4 (k): k_route occupancy A/B (waves_per_eu 8 with 12 VGPRs spilled vs 4 without),
# bench + kernel trace per variant.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4k}
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
summ() { python -c "
import json,sys; s=open('$1').read(); d=json.loads(s[s.index('{'):])
print('$2', round(d['value']/1e6,2), 'M p50', round(d['p50_latency_ms'],3), 'ms/step', round(d['ms_per_step'],3))"; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base wpe4; do
  if [ $v = wpe4 ]; then export CHANAMQ_DP_SO=$GRAFT_REPO_ROOT/chanamq_amd/ops/_dataplane_wpe4.so; fi
  timeout -k 10 120 python bench.py --steps 200 --warmup 5 --soak-s 0 --chunk 32768 > $O/bench_$v.json 2> $O/bench_$v.err
  rc=$?; fatal $rc bench; summ $O/bench_$v.json "$v K=200"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t_$v -o run -- python3 bench.py --steps 40 --warmup 5 --soak-s 0 --chunk 32768 > $O/trace_$v.log 2>&1
  rc=$?; fatal $rc trace
  f=$(find $O/t_$v -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp $f $O/kernel_stats_$v.csv && grep -E "k_route\b|k_route\"|Name" $O/kernel_stats_$v.csv | cut -c1-200
  rm -rf $O/t_$v
done
unset CHANAMQ_DP_SO
timeout -k 10 900 python -u -m pytest tests/test_gpu_dataplane.py tests/test_gpu_broker.py -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest.log; tail -3 $O/pytest.log | grep -E "passed|failed"; fatal $rc pytest
timeout -k 10 300 python -u bench/gpu_server_e2e.py --io-threads 8 --wal-soak 30 --out $O/e2e_config4_soak30.json > $O/e2e_config4_soak.log 2>&1
rc=$?; fatal $rc soak; grep "^{" $O/e2e_config4_soak.log | cut -c1-700 | tail -1
exit 0
