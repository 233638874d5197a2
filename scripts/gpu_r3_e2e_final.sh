#!/bin/bash
# Round 3, final tree: the pipelined sharded server at world 4 (four rank processes on this
# GPU, shared-memory exchange; consumers on the owning rank, then through device links),
# and a 30 s config-2 TCP soak at 8 IO threads with the post-load leak check.
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_e2e_final; mkdir -p $O
timeout -k 10 500 python -u bench/gpu_server_e2e.py --sharded 4 --seconds 4 --io-threads 2 --only config2 --paced 0 \
  --out $O/sharded_w4_config2.json > $O/sharded_w4.log 2>&1
rc=$?; tail -3 $O/sharded_w4.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u bench/gpu_server_e2e.py --seconds 30 --io-threads 8 --only config2 --paced 0 \
  --out $O/config2_soak30s_io8.json > $O/soak.log 2>&1
rc=$?; tail -3 $O/soak.log | cut -c1-400; exit $rc
