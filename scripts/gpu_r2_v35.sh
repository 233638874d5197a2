set -o pipefail
O=gpurun_out/r2_v35; mkdir -p $O
timeout -k 10 400 python -u bench/gpu_server_e2e.py --only config5 --seconds 4 --io-threads 2 --paced 0 --out $O/e2e_config5.json > $O/e2e.log 2>&1 || { tail -30 $O/e2e.log; exit 1; }
python -c "
import json; r=json.load(open('$O/e2e_config5.json'))['results'][0]
print({k: r[k] for k in ('recv_msgs_per_s','sent_msgs_per_s','p50_us','redelivered','requeued','flow_off','flow_off_server')})
for t in r['timeline']: print(t)
"
