set -o pipefail
O=gpurun_out/r2_v36; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 400 python -u bench/gpu_server_e2e.py --only config5 --seconds 4 --io-threads 2 --out $O/e2e_config5.json > $O/e2e.log 2>&1 || { tail -30 $O/e2e.log; exit 1; }
python -c "
import json; rs=json.load(open('$O/e2e_config5.json'))['results']
for r in rs: print({k: r.get(k) for k in ('recv_msgs_per_s','sent_msgs_per_s','p50_us','p99_us','redelivered','requeued','flow_off','flow_off_server','rate_per_producer')})
r=rs[0]
for t in r['timeline'][::4]: print(t)
"
timeout -k 10 240 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
