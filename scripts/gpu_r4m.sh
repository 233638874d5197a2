#!/bin/bash
# Round 4 (m): config 4 vs group delay / IO threads; sharded config 2 (2 ranks on this GPU)
# with consumers local vs on the other rank (device links).
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4m}
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
for cfg in "4 8" "5 8" "3 4" "6 8"; do
  set -- $cfg
  timeout -k 10 300 python -u bench/gpu_server_e2e.py --seconds 4 --io-threads $2 --only config4 --paced 0 \
    --persist-group-ms $1 --out $O/e2e_config4_g$1_io$2.json > $O/e2e_config4_g$1_io$2.log 2>&1
  rc=$?; fatal $rc e2e4; python -c "
import json; d=json.load(open('$O/e2e_config4_g$1_io$2.json')); r=(d['results'] if isinstance(d,dict) else d)[0]
s=r['store'] or {}; b=r.get('body_log') or {}
print('group $1 ms io $2: config4', round(r['confirmed_per_s']/1e6,3), 'M/s p50', r['p50_us'], 'commits', s.get('commits'), 'body GB', round(b.get('written',0)/1e9,2), 'busy', round(s.get('busy_s',0),2), r.get('thread_cpu_s'))"
done
timeout -k 10 600 python -u bench/gpu_server_e2e.py --seconds 4 --sharded 2 --only config2 --paced 0 --io-threads 4 \
  --out $O/e2e_sharded2_config2.json > $O/e2e_sharded2.log 2>&1
rc=$?; fatal $rc sharded; grep "^{" $O/e2e_sharded2.log | cut -c1-300
exit 0
