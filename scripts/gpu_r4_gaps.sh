#!/bin/bash
# Round 4: kernel durations and launch gaps per step of the headline bench at two step sizes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4_gaps}; mkdir -p $O
for ch in ${CHUNKS:-32768 4096}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t$ch -o run -- python3 bench.py --steps 40 --warmup 5 --soak-s 0 --chunk $ch $EXTRA > $O/t$ch.log 2>&1 || { tail -20 $O/t$ch.log; exit 1; }
  python3 scripts/step_gaps.py $O/t$ch > $O/gaps_c$ch.csv; cat $O/gaps_c$ch.csv
  rm -rf $O/t$ch
done
