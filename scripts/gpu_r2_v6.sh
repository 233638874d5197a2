set -o pipefail
O=gpurun_out/r2_v6; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py -m gpu -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench/gpu_server_e2e.py --seconds 3 --io-threads 2,4 --only config2 --out $O/e2e_config2.json > $O/e2e_config2.log 2>&1 || exit $?
grep '^{' $O/e2e_config2.log | cut -c1-330
timeout -k 10 200 python -u bench/gpu_server_e2e.py --seconds 3 --io-threads 4 --only config4 --paced 0 --out $O/e2e_config4.json > $O/e2e_config4.log 2>&1 || exit $?
grep '^{' $O/e2e_config4.log | cut -c1-600
exit $rc
