set -o pipefail
O=gpurun_out/r2_v33; mkdir -p $O
timeout -k 10 400 python -u bench/gpu_server_e2e.py --only config5 --seconds 4 --io-threads 2 --out $O/e2e_config5.json > $O/e2e.log 2>&1 || { tail -30 $O/e2e.log; exit 1; }
cut -c1-1500 $O/e2e.log
