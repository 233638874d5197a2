# Round 2 v3: all GPU tests, then TCP e2e (config 2 at 2/4 IO threads, direct, config 4)
set -o pipefail
O=gpurun_out/r2_v3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench/gpu_server_e2e.py --seconds 3 --io-threads 2,4 --only config2 --out $O/e2e_config2.json > $O/e2e_config2.log 2>&1 || exit $?
tail -6 $O/e2e_config2.log
timeout -k 10 200 python -u bench/gpu_server_e2e.py --seconds 3 --io-threads 4 --only config4 --paced 0 --out $O/e2e_config4.json > $O/e2e_config4.log 2>&1 || exit $?
tail -2 $O/e2e_config4.log
exit $rc
