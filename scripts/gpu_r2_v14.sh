set -o pipefail
O=gpurun_out/r2_v14; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_remote_consume.py tests/test_gpu_sharded.py tests/test_sharded_server.py tests/test_gpu_broker.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -3
