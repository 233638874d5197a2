set -o pipefail
O=gpurun_out/r2_v32; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_remote_consume.py tests/test_sharded_server.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -60 $O/gpu_tests.log; exit 1; }
tail -12 $O/gpu_tests.log
