cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python dbg_phase.py > gpurun_out/phase.log 2>&1
timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/bench3.log 2>&1
echo "bench exit $?" >> gpurun_out/bench3.log
