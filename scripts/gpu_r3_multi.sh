#!/bin/bash
# Round 3: BASELINE configs 3 and 5 on one GPU (bench.py workloads), then the 8-rank
# multi-process path of bench.py (the driver's N=8 code path, exchange staged through gloo
# because RCCL refuses several ranks on one device) with all 8 ranks sharing this GPU.
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_multi; mkdir -p $O
timeout -k 10 180 python bench.py --workload fanout --steps 20 --warmup 5 --soak-s 0 > $O/bench_config3_fanout.json 2> $O/bench_config3.err
rc=$?; [ $rc -ne 0 ] && exit $rc
timeout -k 10 180 python bench.py --workload storm --steps 40 --warmup 8 --soak-s 0 > $O/bench_config5_storm.json 2> $O/bench_config5.err
rc=$?; [ $rc -ne 0 ] && exit $rc
CHANAMQ_BENCH_BACKEND=gloo timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 8 --steps 10 --warmup 3 --soak-s 0 \
  > $O/bench_8rank_gloo_one_gpu.json 2> $O/bench_8rank_gloo.err
rc=$?; echo "8rank exit $rc" >> $O/bench_8rank_gloo.err; tail -3 $O/bench_8rank_gloo.json | cut -c1-600; exit $rc
