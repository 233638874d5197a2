# Full GPU test suite, then the per-rank-step kernel profile at world 1 / 8 and a 1-GPU
# bench.py run (each step under its own time limit; the first failure ends the call).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r3_suite}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { tail -60 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
RUN=${RUN:-r3_suite} bash scripts/gpu_world_prof.sh || exit 1
timeout -k 10 300 python3 bench.py --steps 40 --warmup 10 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -2 $O/bench.log
if [ -n "$E2E" ]; then
  timeout -k 10 300 python3 -u bench/gpu_server_e2e.py --only "$E2E" --io-threads ${IOT:-4} --seconds 4 \
    --out $O/e2e.json > $O/e2e.log 2>&1 || { tail -30 $O/e2e.log; exit 1; }
  cut -c1-400 $O/e2e.log | grep name
fi
