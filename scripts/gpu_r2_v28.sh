set -o pipefail
O=gpurun_out/r2_v28; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU --kernel-include-regex "k_frame_scan|k_decode|k_store|k_scan" --output-format csv -d $O/pmc -o run -- python3 bench.py --steps 5 --warmup 2 > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
find $O/pmc -name "*counter_collection*" | head -3
