#!/bin/bash
# Round 4 (o): config 4 vs group delay x confirm-read (bytes a confirm-mode connection
# contributes per step), with the copier thread in place.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4o}
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
for cfg in "1 131072" "2 262144" "1 262144" "2 524288" "1.5 196608"; do
  set -- $cfg
  timeout -k 10 300 python -u bench/gpu_server_e2e.py --seconds 4 --io-threads 8 --only config4 --paced 0 \
    --persist-group-ms $1 --confirm-read $2 --out $O/e2e_config4_g$1_cr$2.json > $O/e2e_config4_g$1_cr$2.log 2>&1
  rc=$?; fatal $rc e2e4; python -c "
import json; d=json.load(open('$O/e2e_config4_g$1_cr$2.json')); r=(d['results'] if isinstance(d,dict) else d)[0]
s=r['store'] or {}; b=r.get('body_log') or {}
print('group $1 ms confirm-read $2: config4', round(r['confirmed_per_s']/1e6,3), 'M/s p50', r['p50_us'], 'body GB', round(b.get('written',0)/1e9,2), 'busy', round(s.get('busy_s',0),2), r.get('thread_cpu_s'))"
done
exit 0
