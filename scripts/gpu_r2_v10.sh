set -o pipefail
O=gpurun_out/r2_v10; mkdir -p $O
timeout -k 10 400 python -u bench/gpu_server_e2e.py --seconds 3 --io-threads 2,4 --only config2 --out $O/e2e.json > $O/e2e.log 2>&1 || exit $?
python -c "
import json
for r in json.load(open('$O/e2e.json'))['results']:
    fe=r.get('front_end') or {}
    print(r['io_threads'], round(r.get('rate_per_producer') or 0), 'recv', round(r['recv_msgs_per_s']), 'sent', round(r['sent_msgs_per_s']), 'p50', r['p50_us'], 'flow_off', r.get('flow_off'), {k: fe.get(k) for k in ('dropped_nomem','routed','delivered','log_used','live_msgs')})"
