#!/bin/bash
# round 3: lone-chain speed before / after the first-G change (same box, alternating)
mkdir -p gpurun_out/r3chain
for r in 1 2; do for v in prev new; do
  PFSCDC_LIB=build_ab/lib_$v.so timeout -k 10 120 python tools/chain_latency.py 67108864 2.35 1,16 > gpurun_out/r3chain/${v}_$r.txt 2>&1 || { cat gpurun_out/r3chain/${v}_$r.txt; exit 1; }
  echo "$v $r: $(cat gpurun_out/r3chain/${v}_$r.txt | tr '\n' ' ')"
done; done
