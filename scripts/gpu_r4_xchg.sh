#!/bin/bash
# Round 4: the bench's engine-native exchange -- the one-rank RCCL communicator test, then
# the 2- and 4-rank rehearsal on this one GPU (gloo launcher group => shared-memory
# backend) next to the torch exchange, with the host's per-step exchange times.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4_xchg}
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_sharded.py -m gpu -x -v -k rccl_single --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_rccl.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest_rccl.log; tail -3 $O/pytest_rccl.log; [ $rc -ne 0 ] && exit $rc
for n in 2 4; do
  for x in native torch; do
    CHANAMQ_BENCH_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 30 --warmup 5 --soak-s 0 --xchg $x $EXTRA > $O/bench_${n}r_$x.json 2> $O/bench_${n}r_$x.err
    rc=$?; [ $rc -ne 0 ] && { tail -20 $O/bench_${n}r_$x.err; exit $rc; }
    python -c "import json; d=json.load(open('$O/bench_${n}r_$x.json')); print($n, '$x', round(d['value']/1e6,2), 'M', d['p50_latency_ms'], d['ms_per_step'], d['host_us_per_step'])"
  done
done
