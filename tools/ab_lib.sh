# Same-box A/B of two builds (PFSCDC_LIB), alternating: c2 headline and c4, hash/scan ms.
# usage: bash tools/ab_lib.sh <a.so> <b.so> <reps>
mkdir -p gpurun_out/ablib
A=$1; B=$2; R=${3:-2}
for i in $(seq 1 $R); do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    PFSCDC_LIB=$lib timeout -k 10 200 python bench.py --steps 6 --warmup 2 --no-e2e --no-cpu-baseline > gpurun_out/ablib/c2_${v}_$i.json 2>/dev/null || exit 1
    PFSCDC_LIB=$lib timeout -k 10 200 python bench.py --config c4 --steps 2 --warmup 1 --no-e2e --no-cpu-baseline > gpurun_out/ablib/c4_${v}_$i.json 2>/dev/null || exit 1
  done
done
for f in gpurun_out/ablib/*.json; do python -c "
import json
d=json.load(open('$f')); k=d['kernel_ms']; print('$f', d['value'], round(k['scan'],2), round(k['hash'],2))"; done
