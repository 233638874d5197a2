#!/bin/bash
# Hardware counters per kernel of the one-GPU headline step (bench/world_rehearsal.py
# --world 1), one rocprofv3 --pmc pass per counter group, each under its own time limit:
# two SQ groups (wave cycles, instruction mix, LDS bank conflicts) and the L2 fetch / write
# sizes (FETCH_SIZE alone: it takes 3 of the 4 TCC counters).  Output: gpurun_out/r3_pmc_w1/
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_pmc_w1; mkdir -p $O
k=0
for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "FETCH_SIZE" "WRITE_SIZE"; do
  k=$((k+1))
  timeout -s KILL 150 rocprofv3 --pmc $G --output-format csv -d $O/p$k -o run -- python3 bench/world_rehearsal.py --world 1 --steps 4 --warmup 1 > $O/p$k.log 2>&1 || { tail -20 $O/p$k.log; exit 1; }
  python3 scripts/pmc_summary.py $O/p$k > $O/pmc$k.csv && cat $O/pmc$k.csv
  rm -rf $O/p$k
done
