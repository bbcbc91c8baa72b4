mkdir -p gpurun_out/uw2
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fileset.py > gpurun_out/uw2/t.log 2>&1 || exit 1
for inf in 8589934592 4294967296 2147483648; do
  PFSCDC_UW_INFLIGHT=$inf PFSCDC_TRACE=1 timeout -k 10 600 python bench.py --path uw --config c4 --uw-bytes 17179869184 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/uw2/c4_$inf.json 2> gpurun_out/uw2/c4_$inf.err || exit 1
done
tail -2 gpurun_out/uw2/t.log
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/uw2/*.json")):
    d = json.load(open(f)); print(f.split("/")[-1], d["value"], d["split_ms"])
PY
