cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_dataplane.py -m gpu -x -q > gpurun_out/gpu_tests_dp.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/gpu_tests_dp.log; tail -2 gpurun_out/gpu_tests_dp.log
[ $rc -eq 0 ] || exit $rc
for v in blit sdma; do
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 --copy-engine $v > gpurun_out/copy2_$v.json 2>gpurun_out/copy2_$v.err || exit $?
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/copy2_$v.json'));print(round(d['value']/1e6,2), round(d['ms_per_step'],3))")"
done
