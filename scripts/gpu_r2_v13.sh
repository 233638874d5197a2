set -o pipefail
O=gpurun_out/r2_v13; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dataplane.py tests/test_gpu_ids.py > $O/dp_tests.log 2>&1 || { tail -30 $O/dp_tests.log; exit 1; }
tail -3 $O/dp_tests.log
timeout -k 10 300 python -u bench/gpu_server_e2e.py --seconds 3 --io-threads 2 --only config2 --paced 0 --out $O/e2e.json > $O/e2e.log 2>&1 || exit $?
python -c "
import json
for r in json.load(open('$O/e2e.json'))['results']:
    fe=r.get('front_end') or {}
    print(r['io_threads'], 'recv', round(r['recv_msgs_per_s']), 'sent', round(r['sent_msgs_per_s']), 'flow_off', r.get('flow_off'))
    print(json.dumps(r['after']))
    print({k: fe.get(k) for k in ('dropped_nomem','routed','delivered','log_used','live_msgs','ring_full','unroutable','expired')})"
