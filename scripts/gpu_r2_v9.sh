set -o pipefail
O=gpurun_out/r2_v9; mkdir -p $O
timeout -k 10 200 python -u bench/gpu_server_e2e.py --seconds 3 --io-threads 2 --only config2 --paced 0 --out $O/e2e.json > $O/e2e.log 2>&1 || exit $?
python -c "
import json; r=json.load(open('$O/e2e.json'))['results'][0]; print(r['recv_msgs_per_s'], r['sent_msgs_per_s'], r['flow_off'], r['front_end'])"
