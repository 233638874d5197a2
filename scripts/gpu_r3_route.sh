#!/bin/bash
# Round 3: GPU suite on the tree under test, per-GPU kernel time at world 1 / 8, headline
# bench at the driver's K/W, config-2 TCP IO-thread sweep 1/2/4/8 (unpaced + paced 50%).
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r3_route}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
RUN=${RUN:-r3_route} bash scripts/gpu_world_prof.sh > $O/world.log 2>&1
rc=$?; grep -E "TOTAL" $O/world.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20.json 2> $O/bench_k20.err
rc=$?; [ $rc -ne 0 ] && exit $rc
if [ -n "$FS" ]; then
  timeout -k 10 200 python scripts/frame_scan_phases.py > $O/frame_scan_phases.txt 2>&1
  rc=$?; cat $O/frame_scan_phases.txt | tail -14; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$E2E" ]; then
  timeout -k 10 600 python -u bench/gpu_server_e2e.py --seconds 4 --io-threads 1,2,4,8 --only config2 --paced 0.5 \
    --out $O/e2e_config2_io_sweep.json > $O/e2e_sweep.log 2>&1
  rc=$?; tail -4 $O/e2e_sweep.log | cut -c1-400; exit $rc
fi
