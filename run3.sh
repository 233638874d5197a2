cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench1.log 2>&1
rc=$?; echo "bench exit $rc" >> gpurun_out/bench1.log
exit $rc
