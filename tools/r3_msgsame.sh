#!/bin/bash
# round 3 (timing only): is a lone chain waiting on its message loads?  The same chains with
# every fast block loading the segment's first block (L2-resident) instead of block blk+2
mkdir -p gpurun_out/r3ms
for r in 1 2; do for v in new msgsame; do
  PFSCDC_LIB=build_ab/lib_$v.so timeout -k 10 120 python tools/chain_latency.py 67108864 2.35 1,16,4096 > gpurun_out/r3ms/${v}_$r.txt 2>&1 || { cat gpurun_out/r3ms/${v}_$r.txt; exit 1; }
  echo "$v $r: $(grep chains gpurun_out/r3ms/${v}_$r.txt | tr '\n' ' ')"
done; done
