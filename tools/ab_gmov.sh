# A/B of the move-form G round (libpfscdc_mov.so, -DPFS_G_MOVES) against the DPP-fold form
mkdir -p gpurun_out/gmov
PFSCDC_LIB=$PWD/pfs_amd/libpfscdc_mov.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_refid.py > gpurun_out/gmov/t.log 2>&1 || { tail -20 gpurun_out/gmov/t.log; exit 1; }
for rep in 1 2; do for lib in libpfscdc.so libpfscdc_mov.so; do
  PFSCDC_LIB=$PWD/pfs_amd/$lib timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/gmov/c2_${lib}_$rep.json 2>/dev/null || exit 1
  PFSCDC_LIB=$PWD/pfs_amd/$lib timeout -k 10 300 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/gmov/c4_${lib}_$rep.json 2>/dev/null || exit 1
done; done
for lib in libpfscdc.so libpfscdc_mov.so; do
  PFSCDC_LIB=$PWD/pfs_amd/$lib timeout -k 10 300 python bench.py --path commit --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/gmov/commit_${lib}.json 2>/dev/null || exit 1
  PFSCDC_LIB=$PWD/pfs_amd/$lib timeout -k 10 300 python bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/gmov/c3_${lib}.json 2>/dev/null || exit 1
done
tail -2 gpurun_out/gmov/t.log
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/gmov/*.json")):
    d = json.load(open(f)); k = d["kernel_ms"]
    print(f.split("/")[-1], d["value"], round(k["hash"], 1), round(k.get("create", 0), 1))
PY
