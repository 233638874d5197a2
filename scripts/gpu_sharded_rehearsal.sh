# 2 ranks of the sharded bench on ONE GPU (gloo exchange staged through the host):
# rehearses bench.py's multi-GPU code path where only one MI355X is available.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export CHANAMQ_BENCH_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29611 bench.py --gpus 2 --steps 20 --warmup 5 --producers 64 > gpurun_out/shard_rehearsal.log 2>&1
rc=$?; echo "rehearsal exit $rc" >> gpurun_out/shard_rehearsal.log
exit $rc
