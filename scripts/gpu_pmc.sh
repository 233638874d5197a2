# Hardware counters per kernel of the sharded rehearsal step (one rocprofv3 --pmc pass per
# counter group, each under its own time limit).  Output: gpurun_out/$RUN/pmc<k>.csv
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r3_pmc}; mkdir -p $O
W=${W:-8}
k=0
for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
  k=$((k+1))
  timeout -s KILL 150 rocprofv3 --pmc $G --output-format csv -d $O/p$k -o run -- python3 bench/world_rehearsal.py --world $W --steps 4 --warmup 1 > $O/p$k.log 2>&1 || { tail -20 $O/p$k.log; exit 1; }
  python3 scripts/pmc_summary.py $O/p$k > $O/pmc$k.csv && cat $O/pmc$k.csv
  rm -rf $O/p$k
done
