# Pipelined sharded server on one GPU (2-3 ranks, shared-memory exchange), then the GPU suite.
set -o pipefail
O=gpurun_out/${RUN:-r3_sfe}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded_server.py -v -s --timeout 400 --timeout-method thread > $O/sharded_fe.log 2>&1
rc=$?; grep -E "PASSED|FAILED|Error|assert" $O/sharded_fe.log | tail -30 | cut -c1-300
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -5 $O/gpu_tests.log; exit $rc
