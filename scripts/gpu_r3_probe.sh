# Round 3 probe: config-5 TCP storm alone (set-up timeout of the r2 final tree), then the GPU suite.
set -o pipefail
O=gpurun_out/${RUN:-r3_probe}; mkdir -p $O
timeout -k 10 240 python -u bench/gpu_server_e2e.py --seconds 3 --io-threads 4 --only config5 --paced 0 --out $O/e2e_config5.json > $O/e2e_config5.log 2>&1
echo "config5 rc=$?"; tail -5 $O/e2e_config5.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -5 $O/gpu_tests.log
exit $rc
