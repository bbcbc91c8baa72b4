# A/B of the hash-kernel wave priority knob (PFSCDC_HASH_PRIO, remaining blocks) on the commit
# path (long chunk chains) and the headline put path.
mkdir -p gpurun_out/prio
for v in "$@"; do
  PFSCDC_HASH_PRIO=$v timeout -k 10 300 python bench.py --path commit --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prio/commit_$v.json 2> gpurun_out/prio/commit_$v.err || exit 1
  PFSCDC_HASH_PRIO=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/prio/put_$v.json 2> gpurun_out/prio/put_$v.err || exit 1
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/prio/*.json")):
    d = json.load(open(f))
    print(f.split("/")[-1], d["value"], d["kernel_ms"])
PY
