# egress D2H on different SDMA engines (H2D stays on the runtime's engine)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for e in 1 0 2 3; do
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 --copy-engine sdma --sdma-engine $e > gpurun_out/sdma_$e.json 2>gpurun_out/sdma_$e.err || exit $?
  echo "sdma $e $(python -c "import json;d=json.load(open('gpurun_out/sdma_$e.json'));print(round(d['value']/1e6,2), round(d['ms_per_step'],3))")"
done
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/blit.json 2>gpurun_out/blit.err || exit $?
echo "blit $(python -c "import json;d=json.load(open('gpurun_out/blit.json'));print(round(d['value']/1e6,2), round(d['ms_per_step'],3))")"
