mkdir -p gpurun_out/sprio
for rep in 1 2; do for v in 0 1 2; do
  PFSCDC_SCAN_PRIO=$v timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/sprio/put_${v}_$rep.json 2> gpurun_out/sprio/put_${v}_$rep.err || exit 1
done; done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/sprio/*.json")):
    d = json.load(open(f)); k = d["kernel_ms"]
    print(f.split("/")[-1], d["value"], round(k["hash"], 2), round(k["scan"], 2))
PY
