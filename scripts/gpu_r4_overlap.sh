#!/bin/bash
# Round 4: overlapped steps -- the GPU dataplane/broker/sharded suites (golden byte-exact
# scenarios run on the overlapped engine), then the step-size sweep and a kernel trace.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${RUN:-r4_overlap}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dataplane.py tests/test_gpu_broker.py tests/test_golden_dataplane.py tests/test_gpu_ids.py tests/test_gpu_scale.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest.log; tail -4 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for ch in ${CHUNKS:-65536 49152 32768 24576 16384}; do
  for k in 20 200; do
    timeout -k 10 120 python bench.py --steps $k --warmup 5 --soak-s 0 --chunk $ch $EXTRA > $O/bench_c${ch}_k$k.json 2> $O/bench_c${ch}_k$k.err
    rc=$?; [ $rc -ne 0 ] && { tail -5 $O/bench_c${ch}_k$k.err; exit $rc; }
    python -c "import json,sys; d=json.load(open('$O/bench_c${ch}_k$k.json')); print($ch, $k, round(d['value']/1e6,2), 'M', round(d['p50_latency_ms'],3), round(d['p99_latency_ms'],3), round(d['ms_per_step'],3), d['host_us_per_step'])"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- python3 bench.py --steps 40 --warmup 5 --soak-s 0 --chunk 32768 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
python3 scripts/step_gaps.py $O/t > $O/gaps_c32768.csv; cat $O/gaps_c32768.csv
python3 scripts/timeline.py $O/t > $O/timeline.txt 2>&1; rm -rf $O/t
