mkdir -p gpurun_out/prio6
for rep in 1 2; do for v in 0 8192 4096 16384; do
  PFSCDC_HASH_PRIO=$v timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/prio6/c4_${v}_$rep.json 2> gpurun_out/prio6/c4_${v}_$rep.err || exit 1
done; done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/prio6/*.json")):
    d = json.load(open(f)); k = d["kernel_ms"]
    print(f.split("/")[-1], d["value"], round(k["hash"], 1), round(k["scan"], 1))
PY
