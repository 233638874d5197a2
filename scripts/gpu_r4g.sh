#!/bin/bash
# Round 4 (g): where the K=20 window loses against steady state (trace of the driver's
# K=20/W=5 run at two step sizes; the same with a longer warm-up as a control).
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4g}
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
summ() { python -c "
import json,sys; s=open('$1').read(); d=json.loads(s[s.index('{'):])
print('$2', round(d['value']/1e6,2), 'M p50', round(d['p50_latency_ms'],3), 'ms/step', round(d['ms_per_step'],3), d['host_us_per_step'])"; }
for cfg in "32768 20 5" "32768 20 40" "49152 20 5" "49152 20 40" "65536 20 5" "65536 20 40"; do
  set -- $cfg
  f=$O/bench_c$1_k$2_w$3
  timeout -k 10 120 python bench.py --steps $2 --warmup $3 --soak-s 0 --chunk $1 > $f.json 2> $f.err
  rc=$?; fatal $rc bench; [ $rc -ne 0 ] && { tail -5 $f.err; continue; }
  summ $f.json "chunk $1 K=$2 W=$3"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for ch in 32768 49152; do
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/t$ch -o run -- python3 bench.py --steps 20 --warmup 5 --soak-s 0 --chunk $ch > $O/trace$ch.log 2>&1
  rc=$?; fatal $rc trace
  mkdir -p $O/trace$ch
  for f in $(find $O/t$ch -name "*.csv"); do gzip -c "$f" > $O/trace$ch/$(basename "$f").gz; done
  rm -rf $O/t$ch
done
exit 0
