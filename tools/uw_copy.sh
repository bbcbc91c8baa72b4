mkdir -p gpurun_out/uw3
for t in 1 8 16; do
  PFSCDC_COPY_THREADS=$t PFSCDC_UW_INFLIGHT=17179869184 PFSCDC_TRACE=1 timeout -k 10 600 python bench.py --path uw --config c4 --uw-bytes 34359738368 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/uw3/c4_t$t.json 2> gpurun_out/uw3/c4_t$t.err || exit 1
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/uw3/*.json")):
    d = json.load(open(f)); print(f.split("/")[-1], d["value"], d["split_ms"])
PY
grep pfscdc gpurun_out/uw3/c4_t8.err | tail -3
