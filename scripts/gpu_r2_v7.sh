set -o pipefail
O=gpurun_out/r2_v7; mkdir -p $O
timeout -k 10 500 python -u bench/gpu_server_e2e.py --seconds 3 --io-threads 2 --only config2 --paced 0 --rates 2000000,3000000,4000000,5000000 --out $O/e2e_rates_io2.json > $O/e2e_rates_io2.log 2>&1 || exit $?
grep '^{' $O/e2e_rates_io2.log | cut -c1-700
timeout -k 10 300 python -u bench/gpu_server_e2e.py --seconds 3 --io-threads 4 --only config2 --paced 0 --rates 3000000,5000000 --out $O/e2e_rates_io4.json > $O/e2e_rates_io4.log 2>&1 || exit $?
grep '^{' $O/e2e_rates_io4.log | cut -c1-700
