set -o pipefail
O=gpurun_out/r2_v8; mkdir -p $O
for wb in 8388608 67108864 1073741824; do
timeout -k 10 200 python -u bench/gpu_server_e2e.py --seconds 3 --io-threads 2 --only config2 --paced 0 --wblock-high $wb --out $O/e2e_wb$wb.json > $O/e2e_wb$wb.log 2>&1 || exit $?
grep '^{' $O/e2e_wb$wb.log | cut -c1-200; grep -o '"thread_cpu_s.*' $O/e2e_wb$wb.log
done
