#!/bin/bash
# Round 4 (q): the ~6 ms stalls at some step sizes -- a kernel + memory-copy trace of the
# K=20 run at 40960 (stalls) and 49152 (clean).
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4q}
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for ch in 40960 49152; do
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/t$ch -o run -- python3 bench.py --steps 20 --warmup 5 --soak-s 0 --chunk $ch > $O/trace$ch.log 2>&1
  rc=$?; fatal $rc trace
  grep -o '"value": [0-9.e+]*\|"p99_latency_ms": [0-9.]*' $O/trace$ch.log | tr '\n' ' '; echo
  mkdir -p $O/trace$ch
  for f in $(find $O/t$ch -name "*.csv"); do gzip -c "$f" > $O/trace$ch/$(basename "$f").gz; done
  rm -rf $O/t$ch
done
exit 0
