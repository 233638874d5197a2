set -o pipefail
O=gpurun_out/r2_v22; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu tests/test_gpu_launcher.py > $O/launcher.log 2>&1 || { tail -40 $O/launcher.log; cat /tmp/pytest-of-*/pytest-*/test_gpu_server_default_sizi*/srv.log 2>/dev/null | tail -20; exit 1; }
tail -3 $O/launcher.log
