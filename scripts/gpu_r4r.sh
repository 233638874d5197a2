#!/bin/bash
# Round 4 (r): the K=20 window with the collector off inside it, at the stalling sizes.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4r}
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
i=0
for ch in 40960 45056 49152 65536 49152 40960 32768; do
  i=$((i+1))
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --chunk $ch --soak-s 0 > $O/bench_${i}_c$ch.json 2> $O/bench_${i}_c$ch.err; rc=$?; fatal $rc bench
  python -c "
import json; s=open('$O/bench_${i}_c$ch.json').read(); d=json.loads(s[s.index('{'):])
print('chunk $ch K=20', round(d['value']/1e6,2), 'M p50', round(d['p50_latency_ms'],3), 'p99', round(d['p99_latency_ms'],3))"
done
exit 0
