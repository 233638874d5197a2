# Pipelined sharded server on one GPU (2 ranks, shared-memory exchange), then the GPU suite.
set -o pipefail
O=gpurun_out/${RUN:-r3_sfe}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded_server.py -x -v -s --timeout 300 --timeout-method thread > $O/sharded_fe.log 2>&1
rc=$?; tail -40 $O/sharded_fe.log | cut -c1-300
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -5 $O/gpu_tests.log; exit $rc
