set -o pipefail
O=gpurun_out/r2_v52; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 && tail -2 $O/gpu_tests.log &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -2 $O/smoke.log &&
timeout -k 10 240 python -u bench.py > $O/bench_config2.json 2> $O/c2.err && cat $O/bench_config2.json &&
CHANAMQ_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_2rank_gloo.json 2> $O/g2.err && tail -1 $O/bench_2rank_gloo.json &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_w8 -o run -- python3 bench/world_rehearsal.py --world 8 --steps 16 --warmup 4 > $O/prof_w8.log 2>&1 && grep '"world"' $O/prof_w8.log
