# Sharded pipelined server e2e (2 ranks on one GPU, shm exchange: local vs remote
# consumers), the config-4 WAL soak, and the per-rank-step kernel profile at world 1 / 8.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r3_se2e}; mkdir -p $O
timeout -k 10 420 python3 -u bench/gpu_server_e2e.py --sharded 2 --only ${ONLY:-config2} --seconds 4 \
  --io-threads 2 --out $O/sharded_e2e.json > $O/sharded_e2e.log 2>&1 || { tail -30 $O/sharded_e2e.log; exit 1; }
cat $O/sharded_e2e.log
timeout -k 10 200 python3 -u bench/gpu_server_e2e.py --wal-soak ${SOAK:-60} --out $O/wal_soak.json > $O/wal_soak.log 2>&1 || { tail -30 $O/wal_soak.log; exit 1; }
cat $O/wal_soak.log
[ -n "$NOPROF" ] || RUN=${RUN:-r3_se2e} bash scripts/gpu_world_prof.sh
