#!/bin/bash
# Round 4 (s): ingress in three rotating slots (prefetch never waits on the GPU): the
# stall check at K=20, then the full GPU suite (-x) and smoke.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4s}
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
i=0
for ch in 49152 65536 49152 40960 32768 49152; do
  i=$((i+1))
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --chunk $ch --soak-s 0 > $O/bench_${i}_c$ch.json 2> $O/bench_${i}_c$ch.err; rc=$?; fatal $rc bench
  python -c "
import json; s=open('$O/bench_${i}_c$ch.json').read(); d=json.loads(s[s.index('{'):])
print('chunk $ch K=20', round(d['value']/1e6,2), 'M p50', round(d['p50_latency_ms'],3), 'p99', round(d['p99_latency_ms'],3), d['slowest_iteration'])"
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest_gpu.log; tail -12 $O/pytest_gpu.log | grep -E "passed|failed|FAILED|ERROR"; fatal $rc pytest
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; fatal $rc smoke
exit 0
