set -u -o pipefail
timeout -k 10 600 python bench.py > gpurun_out/full.json 2> gpurun_out/full.err || { tail -5 gpurun_out/full.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/full.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"])
print("png", d["e2e_png"])
print("jpeg", d["e2e_jpeg"])
print("host", d["e2e_host"]["value"], "cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["cores"])
print(d["per_class"])
PY
