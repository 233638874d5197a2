#!/bin/bash
# Round-3 verification on one MI355X: smoke, GPU suite, headline bench at the driver's
# K/W and at K=50, 2-rank gloo rehearsal of the sharded bench (ranks share the GPU).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3v
O=gpurun_out/r3v
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke exit $rc" >> $O/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20.json 2> $O/bench_k20.err
rc=$?; [ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python bench.py --gpus 1 --steps 50 --warmup 10 > $O/bench_k50.json 2> $O/bench_k50.err
rc=$?; [ $rc -ne 0 ] && exit $rc
CHANAMQ_BENCH_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --soak-s 0 > $O/bench_2rank_gloo.json 2> $O/bench_2rank_gloo.err
rc=$?; echo "2rank exit $rc" >> $O/bench_2rank_gloo.err; [ $rc -ne 0 ] && exit $rc
# kernel statistics of the headline bench itself (rocprofv3 --kernel-trace --stats)
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 20 --warmup 5 --soak-s 0 > $O/prof.log 2>&1
echo "prof exit $?" >> $O/prof.log
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/bench_kernel_stats.csv \;
