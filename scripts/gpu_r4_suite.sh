#!/bin/bash
# Round 4: the driver's GPU tier as it runs it (one pytest process, -x), then smoke and
# the headline bench at the driver's K/W.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4_suite}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest_gpu.log; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke exit $rc" >> $O/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20.json 2> $O/bench_k20.err
rc=$?; cat $O/bench_k20.json; exit $rc
