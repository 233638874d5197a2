set -o pipefail
O=gpurun_out/r2_v53; mkdir -p $O
timeout -k 10 900 python -u bench/gpu_server_e2e.py --seconds 4 --io-threads 2 --paced 0.5 --out $O/e2e_all_specs_final.json > $O/e2e.log 2>&1 || { tail -30 $O/e2e.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r2_v53/e2e_all_specs_final.json"))
print(json.dumps(d)[:3000])
PY
