# egress copy-engine sweep + per-step timeline of the sdma variant
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in blit sdma nocu; do
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 --copy-engine $v > gpurun_out/copy3_$v.json 2>gpurun_out/copy3_$v.err || exit $?
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/copy3_$v.json'));print(round(d['value']/1e6,2), round(d['ms_per_step'],3))")"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof_sdma -o run -- python3 bench.py --steps 20 --warmup 5 --copy-engine sdma > gpurun_out/prof_sdma.log 2>&1
echo "prof exit $?"
