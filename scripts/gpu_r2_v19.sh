set -o pipefail
O=gpurun_out/r2_v19; mkdir -p $O
timeout -k 10 600 python -u bench/gpu_server_e2e.py --seconds 4 --io-threads 2 --paced 0.5 --out $O/e2e.json > $O/e2e.log 2>&1 || { tail -30 $O/e2e.log; exit 1; }
python -c "
import json
for r in json.load(open('$O/e2e.json'))['results']:
    fe=r.get('front_end') or {}
    print(r['name'], r['io_threads'], 'rate', r.get('rate_per_producer'), 'recv', round(r['recv_msgs_per_s']), 'sent', round(r['sent_msgs_per_s']), 'conf', round(r.get('confirmed_per_s') or 0), 'p50', r['p50_us'], 'p99', r['p99_us'], 'err', r.get('error'), 'store', r.get('store'))"
timeout -k 10 120 python -u bench/persist_worker_bench.py --steps 200 --window 16 --fsync > $O/persist_w16.json 2>&1 && cat $O/persist_w16.json
