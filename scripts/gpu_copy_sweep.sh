# egress D2H copy strategy sweep on the headline bench (see engine.hip copy_engine)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/gpu_tests.log; tail -2 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for v in "kernel 8" "kernel 16" "kernel 32" "kernel 64" "blit 16"; do
  set -- $v
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 --copy-engine $1 --copy-wgs $2 > gpurun_out/copy_$1_$2.json 2>gpurun_out/copy_$1_$2.err || exit $?
  echo "$1 $2 $(python -c "import json;d=json.load(open('gpurun_out/copy_$1_$2.json'));print(round(d['value']/1e6,2), round(d['ms_per_step'],3))")"
done
DEBUG_CLR_LIMIT_BLIT_WG=16 timeout -k 10 200 python bench.py --steps 50 --warmup 10 --copy-engine blit > gpurun_out/copy_blitlim.json 2>gpurun_out/copy_blitlim.err || exit $?
echo "blit+limit16 $(python -c "import json;d=json.load(open('gpurun_out/copy_blitlim.json'));print(round(d['value']/1e6,2), round(d['ms_per_step'],3))")"
