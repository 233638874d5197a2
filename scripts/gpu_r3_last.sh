#!/bin/bash
# Round 3, last tree: GPU suite, kernel chain at world 1 / 8, headline bench, config 4 and
# config 2 over TCP at the default per-connection reads (confirm-mode connections capped at
# 128 KiB), k_route's L2->HBM write bytes (PMC WRITE_SIZE).
cd $GRAFT_REPO_ROOT
RUN=r3_last bash scripts/gpu_r3_route.sh || exit $?
O=gpurun_out/r3_last
for spec in config4 config2; do
  timeout -k 10 200 python -u bench/gpu_server_e2e.py --seconds 5 --io-threads 8 --only $spec --paced 0 \
    --out $O/e2e_$spec.json > $O/e2e_$spec.log 2>&1
  rc=$?; tail -1 $O/e2e_$spec.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pw -o run -- python3 bench/world_rehearsal.py --world 1 --steps 4 --warmup 1 > $O/pw.log 2>&1 || exit 1
python3 scripts/pmc_summary.py $O/pw > $O/pmc_write_size.csv && head -6 $O/pmc_write_size.csv
rm -rf $O/pw
