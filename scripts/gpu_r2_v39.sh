set -o pipefail
O=gpurun_out/r2_v39; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_broker_soak.py -m gpu -x -v -s --timeout 200 --timeout-method thread > $O/soak.log 2>&1 || { tail -40 $O/soak.log; exit 1; }
grep -E "soak:|PASSED|FAILED" $O/soak.log
