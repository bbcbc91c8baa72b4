mkdir -p gpurun_out/prio7
timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/prio7/c2_auto.json 2> gpurun_out/prio7/c2.err && \
timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/prio7/c4_auto.json 2> gpurun_out/prio7/c4.err && \
timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/prio7/c5_auto.json 2> gpurun_out/prio7/c5.err && \
timeout -k 10 300 python bench.py --path commit --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prio7/commit_c2_auto.json 2> gpurun_out/prio7/cc2.err || exit 1
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/prio7/*.json")):
    d = json.load(open(f)); k = d["kernel_ms"]
    print(f.split("/")[-1], d["value"], round(k["hash"], 1), round(k["scan"], 1), round(k.get("create", 0), 1))
PY
