# kernel + memory-copy timeline of the headline bench (sdma egress)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof_tl -o run -- python3 bench.py --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/prof_tl.log 2>&1
echo "prof exit $?"
