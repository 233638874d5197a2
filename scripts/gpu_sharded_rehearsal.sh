# 2 ranks of the sharded bench on ONE GPU (gloo exchange staged through the host):
# rehearses bench.py's multi-GPU code path where only one MI355X is available.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export CHANAMQ_BENCH_BACKEND=gloo
for lag in 1 0; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 2961$lag bench.py --gpus 2 --steps 20 --warmup 5 --producers 64 --exchange-lag $lag \
      > gpurun_out/shard_rehearsal_lag$lag.log 2>&1
  rc=$?; echo "rehearsal lag=$lag exit $rc" >> gpurun_out/shard_rehearsal_lag$lag.log
  [ $rc -eq 0 ] || exit $rc
  grep '^{"metric"' gpurun_out/shard_rehearsal_lag$lag.log | cut -c1-200
done
