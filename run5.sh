cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python dbg_phase.py > gpurun_out/phase.log 2>&1
echo "exit $?" >> gpurun_out/phase.log
