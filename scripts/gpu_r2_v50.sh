set -o pipefail
O=gpurun_out/r2_v50; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 && tail -2 $O/gpu_tests.log &&
timeout -k 10 240 python -u bench.py > $O/bench_config2.json 2> $O/c2.err && cat $O/bench_config2.json &&
timeout -k 10 240 python -u bench.py --workload storm > $O/bench_storm.json 2> $O/s.err && cat $O/bench_storm.json &&
timeout -k 10 240 python -u bench.py --workload fanout > $O/bench_fanout.json 2> $O/f.err && cat $O/bench_fanout.json &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_w8 -o run -- python3 bench/world_rehearsal.py --world 8 --steps 16 --warmup 4 > $O/prof_w8.log 2>&1 && grep '"world"' $O/prof_w8.log &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_w4 -o run -- python3 bench/world_rehearsal.py --world 4 --steps 16 --warmup 4 > $O/prof_w4.log 2>&1 && grep '"world"' $O/prof_w4.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_w1 -o run -- python3 bench.py --steps 20 --warmup 5 > $O/prof_w1.log 2>&1
