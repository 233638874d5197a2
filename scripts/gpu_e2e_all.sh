# Whole-broker e2e over loopback TCP: every spec of bench/gpu_server_e2e.py (unpaced, then
# paced at 50%), one process, as the round-2 final-tree run that lost config 5.
set -o pipefail
O=gpurun_out/${RUN:-r3_e2e}; mkdir -p $O
timeout -k 10 900 python -u bench/gpu_server_e2e.py --seconds 4 --io-threads ${IOT:-4} --paced 0.5 --out $O/e2e_all_specs.json > $O/e2e.log 2>&1
rc=$?; tail -12 $O/e2e.log | cut -c1-600; exit $rc
