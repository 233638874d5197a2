# Round 2: pipelined native front end on the GPU box — GPU-server tests, then the TCP e2e
# bench (config 2 swept over IO threads, the other specs at 4 IO threads).
set -o pipefail
O=gpurun_out/${RUN:-r2_v1}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_broker.py tests/test_gpu_dataplane.py tests/test_gpu_ids.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 420 python -u bench/gpu_server_e2e.py --seconds 3 --io-threads ${IOT:-2,4,8} --only config2 --out $O/e2e_config2.json > $O/e2e_config2.log 2>&1 || exit $?
tail -12 $O/e2e_config2.log
timeout -k 10 300 python -u bench/gpu_server_e2e.py --seconds 3 --io-threads 4 --only direct --out $O/e2e_direct.json > $O/e2e_direct.log 2>&1 || exit $?
tail -6 $O/e2e_direct.log
timeout -k 10 200 python -u bench/gpu_server_e2e.py --seconds 3 --io-threads 4 --only config4 --paced 0 --out $O/e2e_config4.json > $O/e2e_config4.log 2>&1 || exit $?
tail -3 $O/e2e_config4.log
exit $rc
