#!/bin/bash
# Round 4 features on the GPU: broker tests (Basic.Get on the step through the pipelined
# front end, record budget), sharded server (config-sized ranks, 64 MiB cross-rank
# message), the RCCL single-rank native exchange, then config 2 over TCP with and
# without Basic.Get pollers.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4_feat}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_broker.py tests/test_gpu_sharded_server.py tests/test_broker_soak.py -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest.log; tail -4 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_r4_xchg.sh || exit $?
timeout -k 10 300 python -u bench/gpu_server_e2e.py --seconds 4 --io-threads 8 --only config2 --paced 0 --getters 4 \
  --out $O/e2e_config2_getters.json > $O/e2e_getters.log 2>&1
rc=$?; tail -2 $O/e2e_getters.log | cut -c1-600; exit $rc
