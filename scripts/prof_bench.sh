cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1 -o run -- python3 bench.py --steps 20 --warmup 5 ${PROF_ARGS} > gpurun_out/prof1.log 2>&1
rc=$?; echo "prof exit $rc" >> gpurun_out/prof1.log
exit $rc
