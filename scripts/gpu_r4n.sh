#!/bin/bash
# Round 4 (n): rotating store-record slots + the front end's copier thread: config 4 at
# 3 ms group delay, the durable / broker / dataplane GPU tests, the 30 s soak.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4n}
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_dataplane.py tests/test_gpu_broker.py -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest.log; tail -3 $O/pytest.log | grep -E "passed|failed|error"; fatal $rc pytest
for g in 3 2; do
  timeout -k 10 300 python -u bench/gpu_server_e2e.py --seconds 4 --io-threads 8 --only config4 --paced 0 \
    --persist-group-ms $g --out $O/e2e_config4_g$g.json > $O/e2e_config4_g$g.log 2>&1
  rc=$?; fatal $rc e2e4; python -c "
import json; d=json.load(open('$O/e2e_config4_g$g.json')); r=(d['results'] if isinstance(d,dict) else d)[0]
s=r['store'] or {}; b=r.get('body_log') or {}
print('group $g ms: config4', round(r['confirmed_per_s']/1e6,3), 'M/s p50', r['p50_us'], 'commits', s.get('commits'), 'body GB', round(b.get('written',0)/1e9,2), 'busy', round(s.get('busy_s',0),2), r.get('thread_cpu_s'))"
done
timeout -k 10 300 python -u bench/gpu_server_e2e.py --io-threads 8 --wal-soak 30 --out $O/e2e_config4_soak30.json > $O/e2e_config4_soak.log 2>&1
rc=$?; fatal $rc soak; grep "^{" $O/e2e_config4_soak.log | cut -c1-500 | tail -1
exit 0
