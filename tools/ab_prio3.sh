# A/B: priority threshold and graded levels (commit path too)
mkdir -p gpurun_out/prio4
run() { PFSCDC_HASH_PRIO=$1 PFSCDC_HASH_PRIO_GRADED=$2 timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/prio4/put_$1_$2_$3.json 2> gpurun_out/prio4/put_$1_$2_$3.err; }
for rep in 1 2; do
  run 0 0 $rep && run 8192 0 $rep && run 6000 0 $rep && run 10000 0 $rep && run 4096 1 $rep && run 8192 1 $rep || exit 1
done
for g in "0 0" "8192 0" "4096 1"; do
  set -- $g
  PFSCDC_HASH_PRIO=$1 PFSCDC_HASH_PRIO_GRADED=$2 timeout -k 10 300 python bench.py --path commit --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prio4/commit_$1_$2.json 2> gpurun_out/prio4/commit_$1_$2.err || exit 1
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/prio4/*.json")):
    d = json.load(open(f))
    k = d["kernel_ms"]
    print(f.split("/")[-1], d["value"], round(k["hash"], 2), round(k["scan"], 2), round(k.get("create", 0), 1), round(k.get("create_content_hash", 0), 1))
PY
