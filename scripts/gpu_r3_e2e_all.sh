#!/bin/bash
# Round 3 final tree: every bench/gpu_server_e2e.py spec over loopback TCP at 8 IO threads
# (unpaced, then paced at half the unpaced rate).
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_e2e_all; mkdir -p $O
timeout -k 10 900 python -u bench/gpu_server_e2e.py --seconds 4 --io-threads 8 --paced 0.5 --out $O/e2e_all_specs_io8_final.json > $O/e2e.log 2>&1
rc=$?; tail -4 $O/e2e.log | cut -c1-300; exit $rc
