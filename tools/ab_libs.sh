#!/bin/bash
# c2 line over several builds (PFSCDC_LIB), round-robin; per-kernel ms.
# usage: bash tools/ab_libs.sh <reps> lib1.so lib2.so ...
R=$1; shift
N="--steps 6 --warmup 2 --no-e2e --no-cpu-baseline --no-literal --no-pipelined --no-chain-floor"
for i in $(seq 1 $R); do
  for lib in "$@"; do
    PFSCDC_LIB=$lib timeout -k 10 200 python bench.py $N > gpurun_out/abl.json 2>gpurun_out/abl.err || { tail -3 gpurun_out/abl.err; exit 1; }
    python -c "
import json
d=json.loads(open('gpurun_out/abl.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('$lib', d['value'], round(k['scan'],3), round(k['hash'],3), flush=True)"
  done
done
