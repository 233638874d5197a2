# Per-GPU kernel time of the headline step at world 1 and 8 (bench/world_rehearsal.py: W
# in-process ranks on one GPU stepped one after another), rocprofv3 kernel trace ->
# kernel time per rank-step (scripts/rank_step_kernels.py; the trace holds warmup + timed steps = 20).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r3_world}; mkdir -p $O
for W in ${WORLDS:-1 8}; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/w$W -o run -- python3 bench/world_rehearsal.py --world $W --steps 16 --warmup 4 > $O/w$W.log 2>&1 || { tail -20 $O/w$W.log; exit 1; }
  db=$(find $O/w$W -name "*.db" | head -1)
  python3 scripts/rank_step_kernels.py $db $((20*W)) $O/w${W}_kernels.csv | tail -80
  rm -rf $O/w$W
done
