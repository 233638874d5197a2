#!/bin/bash
# Round 4 (p): the final tree -- the full GPU suite as the driver runs it (-x), smoke, and
# the K=20 step-size curve around the default.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4p}
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest_gpu.log; tail -12 $O/pytest_gpu.log | grep -E "passed|failed|FAILED|ERROR"; fatal $rc pytest
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; fatal $rc smoke
for ch in 40960 45056 49152 57344 49152; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --chunk $ch > $O/bench_c$ch.json 2> $O/bench_c$ch.err; rc=$?; fatal $rc bench
  python -c "
import json; s=open('$O/bench_c$ch.json').read(); d=json.loads(s[s.index('{'):])
print('chunk $ch K=20', round(d['value']/1e6,2), 'M p50', round(d['p50_latency_ms'],3), 'p99', round(d['p99_latency_ms'],3))"
done
timeout -k 10 120 python bench.py > $O/bench_noflags.json 2> $O/bench_noflags.err; rc=$?; fatal $rc bench; cut -c1-300 $O/bench_noflags.json
exit 0
