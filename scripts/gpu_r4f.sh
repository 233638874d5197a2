#!/bin/bash
# Round 4 (f): config 4 over TCP vs the write-behind's group delay; the sharded-server tests.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4f}
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
for g in ${GROUPS_MS:-0 1 2 3}; do
  timeout -k 10 300 python -u bench/gpu_server_e2e.py --seconds 4 --io-threads 8 --only config4 --paced 0 \
    --persist-group-ms $g --out $O/e2e_config4_g$g.json > $O/e2e_config4_g$g.log 2>&1
  rc=$?; fatal $rc e2e4; python -c "
import json; d=json.load(open('$O/e2e_config4_g$g.json')); r=(d['results'] if isinstance(d,dict) else d)[0]
s=r['store'] or {}; b=r.get('body_log') or {}
print('group $g ms: config4', round(r['confirmed_per_s']/1e6,3), 'M/s p50', r['p50_us'], 'p99', r['p99_us'], 'commits', s.get('commits'), 'body GB', round(b.get('written',0)/1e9,2), 'busy', round(s.get('busy_s',0),2))"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded_server.py -v --timeout 400 --timeout-method thread -p no:cacheprovider > $O/pytest_sharded.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest_sharded.log; tail -3 $O/pytest_sharded.log | grep -E "passed|failed"; fatal $rc pytest
exit 0
