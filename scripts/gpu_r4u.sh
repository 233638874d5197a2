#!/bin/bash
# Round 4 (u): config 2 paced tail with the body tiers' upkeep on / off (spill ring).
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4u}
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
for sp in 0 8589934592 0 8589934592; do
  timeout -k 10 300 python -u bench/gpu_server_e2e.py --seconds 4 --io-threads 8 --only config2 --paced 0.5 --spill-bytes $sp \
    --out $O/e2e_c2_spill$sp.json > $O/e2e_c2_spill$sp.log 2>&1
  rc=$?; fatal $rc e2e; grep "^{" $O/e2e_c2_spill$sp.log | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('spill $sp', d.get('rate_per_producer') and 'paced' or 'unpaced', round(d['recv_msgs_per_s']/1e6,3), 'M p50', round(d['p50_us']), 'p99', round(d['p99_us']))"
done
exit 0
