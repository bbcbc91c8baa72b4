#!/bin/bash
# Same-box A/B of two builds (PFSCDC_LIB): lone-chain latency, c2 line, c4 and c3 hash.
# usage: bash tools/ab_lib2.sh <a.so> <b.so> <reps>
mkdir -p gpurun_out/ablib
A=$1; B=$2; R=${3:-2}
N="--no-e2e --no-cpu-baseline --no-literal --no-pipelined --no-chain-floor"
for i in $(seq 1 $R); do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    PFSCDC_LIB=$lib timeout -k 10 120 python tools/chain_latency.py $((8 << 20)) 2.35 1,4096 > gpurun_out/ablib/cl_${v}_$i.txt 2>/dev/null || exit 1
    PFSCDC_LIB=$lib timeout -k 10 200 python bench.py --steps 6 --warmup 2 $N > gpurun_out/ablib/c2_${v}_$i.json 2>/dev/null || exit 1
    PFSCDC_LIB=$lib timeout -k 10 200 python bench.py --config c4 --steps 2 --warmup 1 $N > gpurun_out/ablib/c4_${v}_$i.json 2>/dev/null || exit 1
    PFSCDC_LIB=$lib timeout -k 10 200 python bench.py --config c3 --steps 2 --warmup 1 $N > gpurun_out/ablib/c3_${v}_$i.json 2>/dev/null || exit 1
    for c in c2 c4 c3; do python -c "
import json
d=json.load(open('gpurun_out/ablib/${c}_${v}_$i.json')); k=d['kernel_ms']; print('$c $v $i', d['value'], round(k['scan'],2), round(k['hash'],2), round(k.get('hash_span',0),2), flush=True)"; done
    grep -h chains gpurun_out/ablib/cl_${v}_$i.txt | sed "s/^/cl $v $i /"
  done
done
