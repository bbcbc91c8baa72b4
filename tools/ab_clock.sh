#!/bin/bash
# c2 line over several builds (PFSCDC_LIB), round-robin: value, scan/hash ms and the clock
# each kernel ran at (MHz, pfscdc_last_kernel_clocks).  usage: bash tools/ab_clock.sh <reps> lib...
R=$1; shift
N="--steps 6 --warmup 2 --no-e2e --no-cpu-baseline --no-literal --no-pipelined --no-chain-floor"
for i in $(seq 1 $R); do
  for lib in "$@"; do
    PFSCDC_LIB=$lib timeout -k 10 200 python bench.py $N > gpurun_out/abc.json 2>gpurun_out/abc.err || { tail -3 gpurun_out/abc.err; exit 1; }
    python -c "
import json
d=json.loads(open('gpurun_out/abc.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('$lib', d['value'], round(k['scan'],3), round(k['hash'],3), round(k.get('scan_mhz',0)), round(k.get('hash_mhz',0)), flush=True)"
  done
done
