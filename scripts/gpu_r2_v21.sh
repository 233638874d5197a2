set -o pipefail
O=gpurun_out/r2_v21; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 240 python -u bench.py > $O/bench_config2.json 2> $O/c2.err || exit 1
cut -c1-330 $O/bench_config2.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 > $O/prof.log 2>&1 || exit 1
export CHANAMQ_BENCH_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 20 --warmup 5 --producers 64 > $O/shard2.log 2>&1 || { tail -20 $O/shard2.log; exit 1; }
grep '^{"metric"' $O/shard2.log | cut -c1-250
