#!/bin/bash
# round 3: the scan's fast-path DMA as buffer_load ... lds (no per-instruction 64-bit address
# add); GPU suite, then same-box A/B against the previous build, alternating
mkdir -p gpurun_out/r3bd
o=gpurun_out/r3bd
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $o/pytest_gpu.log 2>&1 || { tail -30 $o/pytest_gpu.log; exit 1; }
tail -1 $o/pytest_gpu.log
B="--no-cpu-baseline --no-e2e --no-literal --no-pipelined --no-chain-floor"
for r in 1 2 3; do
for v in new buf; do
  PFSCDC_LIB=build_ab/lib_$v.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 $B > $o/c2_${v}_$r.json 2> $o/c2_${v}_$r.err || { tail -5 $o/c2_${v}_$r.err; exit 1; }
  python -c "
import json; d=json.loads(open('$o/c2_${v}_$r.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('c2 $v $r', d['value'], d['ms_per_step'], round(k['scan'],2), round(k['scan_mhz']), round(k['hash'],2), d['roofline']['frac'])"
done
done
