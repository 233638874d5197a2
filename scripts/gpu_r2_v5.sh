set -o pipefail
O=gpurun_out/r2_v5; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; grep -E "FAILED|ERROR" $O/gpu_tests.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python -u bench.py > $O/bench_config2.json 2> $O/bench.err || exit $?
cat $O/bench_config2.json
timeout -k 10 400 python -u bench/gpu_server_e2e.py --seconds 3 --io-threads 2,4 --only config2 --out $O/e2e_config2.json > $O/e2e_config2.log 2>&1 || exit $?
grep '^{' $O/e2e_config2.log | cut -c1-400
exit $rc
