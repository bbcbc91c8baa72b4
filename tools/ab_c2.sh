#!/bin/bash
# Same-box A/B of two builds (PFSCDC_LIB) on the c2 line only, alternating; per-kernel ms.
# usage: bash tools/ab_c2.sh <a.so> <b.so> <reps>
mkdir -p gpurun_out/abc2
N="--steps 8 --warmup 2 --no-e2e --no-cpu-baseline --no-literal --no-pipelined --no-chain-floor"
for i in $(seq 1 ${3:-2}); do
  for v in A B; do
    lib=$1; [ $v = B ] && lib=$2
    PFSCDC_LIB=$lib timeout -k 10 200 python bench.py $N > gpurun_out/abc2/${v}_$i.json 2>gpurun_out/abc2/${v}_$i.err || { tail -3 gpurun_out/abc2/${v}_$i.err; exit 1; }
    python -c "
import json
d=json.loads(open('gpurun_out/abc2/${v}_$i.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('$v', d['value'], d['ms_per_step'], round(k['scan'],3), round(k['select'],3), round(k['hash'],3), round(k['total'],3), flush=True)"
  done
done
