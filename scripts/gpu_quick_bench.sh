# quick headline bench variants (args per line in $VARIANTS, separated by ';')
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
IFS=';' read -ra VS <<< "${VARIANTS:---copy-engine sdma}"
i=0
for v in "${VS[@]}"; do
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 $v > gpurun_out/qb_$i.json 2>gpurun_out/qb_$i.err || { tail -5 gpurun_out/qb_$i.err; exit 1; }
  echo "[$v] $(python -c "import json;d=json.load(open('gpurun_out/qb_$i.json'));print(round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms', d.get('host_us_per_step'))")"
  i=$((i+1))
done
