set -o pipefail
O=gpurun_out/r2_v27; mkdir -p $O
timeout -k 10 900 python -u bench/gpu_server_e2e.py --seconds 8 --io-threads 2,4 --paced 0 --out $O/e2e.json > $O/e2e.log 2>&1 || { tail -30 $O/e2e.log; exit 1; }
python -c "
import json
for r in json.load(open('$O/e2e.json'))['results']:
    a=r.get('after') or {}
    print(r['name'], r['io_threads'], 'recv', round(r['recv_msgs_per_s']), 'sent', round(r['sent_msgs_per_s']), 'p50', round(r['p50_us']), 'leaked', (a.get('leaked') or {}).get('n'), 'live', a.get('live_msgs'), 'queued', a.get('queued_msgs'), 'err', r.get('error'))"
