#!/bin/bash
# Round 4 (v): last check of the final tree -- the full GPU suite (-x, as the driver), smoke,
# and the driver's bench line.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4v}
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest_gpu.log; tail -4 $O/pytest_gpu.log | grep -E "passed|failed|FAILED|ERROR"; fatal $rc pytest
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; fatal $rc smoke
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; rc=$?; fatal $rc bench
python -c "
import json; s=open('$O/bench.json').read(); d=json.loads(s[s.index('{'):])
print('driver line K=20', round(d['value']/1e6,2), 'M p50', round(d['p50_latency_ms'],3), d['slowest_iteration'])"
exit 0
