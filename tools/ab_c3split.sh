#!/bin/bash
# c3 (one 10 GiB stream, two steps in flight): contexts on disjoint CU halves vs shared CUs
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -k "cu_subset or edge" --timeout 100 --timeout-method thread 2>&1 | tail -1
for v in 1 0 1 0 1; do
  timeout -k 10 300 python bench.py --config c3 --steps 4 --warmup 1 --no-cpu-baseline --no-e2e --no-chain-floor --cu-split $v > gpurun_out/c3s_$v.json 2>gpurun_out/c3s_$v.err || { tail -3 gpurun_out/c3s_$v.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/c3s_$v.json').read().strip().splitlines()[-1]); k=d['kernel_ms']; print('cu_split=$v', d['value'], d['ms_per_step'], round(k['scan'],2), round(k['hash'],2), round(k['hash_span'],2), d.get('index_digest'))"
done
