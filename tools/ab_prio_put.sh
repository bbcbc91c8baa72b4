# Repeated A/B of PFSCDC_HASH_PRIO on the headline put path (alternating order).
mkdir -p gpurun_out/prio2
for rep in 1 2; do
  for v in "$@"; do
    PFSCDC_HASH_PRIO=$v timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/prio2/put_${v}_$rep.json 2> gpurun_out/prio2/put_${v}_$rep.err || exit 1
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/prio2/*.json")):
    d = json.load(open(f))
    print(f.split("/")[-1], d["value"], round(d["kernel_ms"]["hash"], 2), round(d["kernel_ms"]["scan"], 2))
PY
