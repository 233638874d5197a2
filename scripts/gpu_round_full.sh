# full GPU pass: tests, headline bench, fanout bench, end-to-end TCP benches, kernel profile
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/gpu_tests.log; tail -2 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --workload fanout > gpurun_out/bench_fanout.json 2> gpurun_out/bench_fanout.err || exit $?
timeout -k 10 300 python bench.py --steps 40 --warmup 10 --workload storm > gpurun_out/bench_storm.json 2> gpurun_out/bench_storm.err || exit $?
cut -c1-300 gpurun_out/bench.json gpurun_out/bench_fanout.json gpurun_out/bench_storm.json
timeout -k 10 400 python bench/gpu_server_e2e.py --seconds 4 --out gpurun_out/gpu_e2e.json > gpurun_out/gpu_e2e.log 2>&1 || exit $?
tail -5 gpurun_out/gpu_e2e.log
bash scripts/prof_bench.sh
