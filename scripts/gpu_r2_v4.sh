set -o pipefail
O=gpurun_out/r2_v4; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -5 $O/gpu_tests.log; grep -E "FAILED|ERROR" $O/gpu_tests.log | head -20
exit $rc
