#!/bin/bash
# Config 4 over TCP (durable, persistent 4 KB, confirms, manual ack): per-connection read per
# step 128 KiB vs 512 KiB at the same 8 IO threads.
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_cfg4_ab; mkdir -p $O
for pcr in 131072 524288; do
  timeout -k 10 200 python -u bench/gpu_server_e2e.py --seconds 5 --io-threads 8 --only config4 --paced 0 \
    --per-conn-read $pcr --out $O/config4_pcr$pcr.json > $O/config4_pcr$pcr.log 2>&1
  rc=$?; tail -2 $O/config4_pcr$pcr.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
done
exit 0
