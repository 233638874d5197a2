set -o pipefail
O=gpurun_out/r2_v23; mkdir -p $O
for ch in 32768 65536 131072; do
  timeout -k 10 240 python -u bench.py --chunk $ch > $O/bench_chunk$ch.json 2> $O/c$ch.err || exit 1
  python -c "import json; r=json.load(open('$O/bench_chunk$ch.json')); print($ch, round(r['value']/1e6,2), 'M/s p50', round(r['p50_latency_ms'],3), 'p99', round(r['p99_latency_ms'],3), 'ms/step', round(r['ms_per_step'],3))"
done
