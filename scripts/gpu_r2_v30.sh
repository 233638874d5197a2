set -o pipefail
O=gpurun_out/r2_v30; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for ch in 32768 65536; do
  timeout -k 10 240 python -u bench.py --chunk $ch > $O/bench_chunk$ch.json 2> $O/c$ch.err || exit 1
  python -c "import json; r=json.load(open('$O/bench_chunk$ch.json')); print($ch, round(r['value']/1e6,2), 'M/s p50', round(r['p50_latency_ms'],3), 'p99', round(r['p99_latency_ms'],3), 'ms/step', round(r['ms_per_step'],3))"
done
timeout -k 10 120 python scripts/frame_scan_phases.py > $O/frame_scan_phases.txt 2>&1 || exit 1
cat $O/frame_scan_phases.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 > $O/prof.log 2>&1 || exit 1
