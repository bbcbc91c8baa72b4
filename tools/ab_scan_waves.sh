# Scan geometry A/B: parity of each build on the GPU, then alternating c2 benches.
# usage: bash tools/ab_scan_waves.sh <reps> <lib>...   (first lib = baseline)
mkdir -p gpurun_out/abw
R=$1; shift
for lib in "$@"; do
  PFSCDC_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/abw/t_$(basename $lib .so).log 2>&1 || { echo "parity FAIL $lib"; exit 1; }
  tail -1 gpurun_out/abw/t_$(basename $lib .so).log
done
for i in $(seq 1 $R); do
  for lib in "$@"; do
    PFSCDC_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 6 --warmup 2 --no-e2e --no-cpu-baseline > gpurun_out/abw/c2_$(basename $lib .so)_$i.json 2>/dev/null || exit 1
  done
done
for f in gpurun_out/abw/*.json; do python -c "
import json
d=json.load(open('$f')); k=d['kernel_ms']; print('$f', d['value'], round(k['scan'],2), round(k['hash'],2), d.get('parity'))"; done
