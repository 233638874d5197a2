#!/bin/bash
# Round 4 (e): the box's disk (what config 4's group commits write to), the sharded-server
# tests, config 2 with Basic.Get pollers (spill on), config 4 with the body-log stats.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4e}
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
{ df -h /tmp; mount | grep -E " /tmp | / " ; lsblk -d -o NAME,ROTA,SIZE,MODEL 2>/dev/null; nproc; } > $O/disk.txt 2>&1
D=$(mktemp -d /tmp/ddtest.XXXX)
for bs in 1M 4M; do
  timeout -k 5 60 dd if=/dev/zero of=$D/f bs=$bs count=$((4096 / ${bs%M})) conv=fdatasync 2>> $O/disk.txt; rm -f $D/f
done
timeout -k 5 60 dd if=/dev/zero of=$D/f bs=1M count=2048 oflag=direct 2>> $O/disk.txt; rm -rf $D
grep -E "copied" $O/disk.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded_server.py -v --timeout 400 --timeout-method thread -p no:cacheprovider > $O/pytest_sharded.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest_sharded.log; tail -3 $O/pytest_sharded.log | grep -E "passed|failed"; fatal $rc pytest
timeout -k 10 400 python -u bench/gpu_server_e2e.py --seconds 4 --io-threads 8 --only config2 --paced 0 --getters 4 \
  --out $O/e2e_config2_getters.json > $O/e2e_config2_getters.log 2>&1
rc=$?; fatal $rc e2e; cut -c1-420 $O/e2e_config2_getters.log | grep "^{" | tail -3
timeout -k 10 300 python -u bench/gpu_server_e2e.py --seconds 4 --io-threads 8 --only config4 --paced 0 \
  --out $O/e2e_config4.json > $O/e2e_config4.log 2>&1
rc=$?; fatal $rc e2e4; python -c "
import json; d=json.load(open('$O/e2e_config4.json')); r=(d['results'] if isinstance(d,dict) else d)[0]
print('config4', round(r['confirmed_per_s']/1e6,3), 'M/s p50', r['p50_us'], r['store'], r.get('body_log'))"
exit 0
