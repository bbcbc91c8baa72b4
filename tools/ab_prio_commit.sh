# A/B of the adaptive hash priority on the commit path (c2, c4) and the put headline
mkdir -p gpurun_out/prio5
for rep in 1 2; do
  for v in adaptive 0; do
    if [ $v = adaptive ]; then unset PFSCDC_HASH_PRIO; else export PFSCDC_HASH_PRIO=$v; fi
    timeout -k 10 300 python bench.py --path commit --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prio5/commit_c2_${v}_$rep.json 2> gpurun_out/prio5/commit_c2_${v}_$rep.err || exit 1
    timeout -k 10 300 python bench.py --path commit --config c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prio5/commit_c4_${v}_$rep.json 2> gpurun_out/prio5/commit_c4_${v}_$rep.err || exit 1
  done
done
unset PFSCDC_HASH_PRIO
timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/prio5/put_adaptive.json 2> gpurun_out/prio5/put_adaptive.err || exit 1
timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/prio5/put_c4_adaptive.json 2> gpurun_out/prio5/put_c4_adaptive.err || exit 1
PFSCDC_HASH_PRIO=0 timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/prio5/put_c4_0.json 2> gpurun_out/prio5/put_c4_0.err || exit 1
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/prio5/*.json")):
    d = json.load(open(f)); k = d["kernel_ms"]
    print(f.split("/")[-1], d["value"], round(k["hash"], 1), round(k.get("create_content_hash", 0), 1), round(k.get("create_ref_id", 0), 1))
PY
