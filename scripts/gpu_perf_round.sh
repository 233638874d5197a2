# GPU tests, then the headline bench with both copy engines, then a kernel-trace profile.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/gpu_tests.log; tail -2 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > gpurun_out/bench_sdma.json 2> gpurun_out/bench_sdma.err || exit $?
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --copy-engine blit > gpurun_out/bench_blit.json 2> gpurun_out/bench_blit.err || exit $?
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --workload fanout > gpurun_out/bench_fanout.json 2> gpurun_out/bench_fanout.err || exit $?
cat gpurun_out/bench_sdma.json gpurun_out/bench_blit.json gpurun_out/bench_fanout.json | cut -c1-400
bash scripts/prof_bench.sh
