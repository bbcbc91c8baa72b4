# A/B: dynamic priority threshold vs static block-parity priority (and both)
mkdir -p gpurun_out/prio3
run() { PFSCDC_HASH_PRIO=$1 PFSCDC_HASH_PRIO_STATIC=$2 timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/prio3/put_$1_$2_$3.json 2> gpurun_out/prio3/put_$1_$2_$3.err; }
for rep in 1 2; do
  run 0 0 $rep && run 8192 0 $rep && run 0 1 $rep && run 8192 1 $rep && run 12000 0 $rep || exit 1
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/prio3/*.json")):
    d = json.load(open(f))
    print(f.split("/")[-1], d["value"], round(d["kernel_ms"]["hash"], 2), round(d["kernel_ms"]["scan"], 2))
PY
