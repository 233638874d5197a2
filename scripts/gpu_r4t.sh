#!/bin/bash
# Round 4 (t): every TCP spec on the final tree, unpaced and paced at 50 % (per-thread CPU
# and front-end stage histograms in the JSON).
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4t}
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u bench/gpu_server_e2e.py --seconds 4 --io-threads 8 --paced 0.5 \
  --out $O/e2e_all_specs_final.json > $O/e2e_all.log 2>&1
rc=$?; fatal $rc e2e; grep "^{" $O/e2e_all.log | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d.get('name'), d.get('rate_per_producer') and 'paced' or 'unpaced', round(d['recv_msgs_per_s']/1e6,3), 'M p50', round(d['p50_us']), 'p99', round(d['p99_us']), d.get('error'))"
exit 0
