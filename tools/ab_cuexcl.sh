#!/bin/bash
# c3 (two steps in flight) and c4 / literal configs[1]: chain-bound scan hashes with one
# workgroup per CU reserved (PFSCDC_HASH_CU_EXCLUSIVE=1, default) vs shareable CUs.
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_configs.py -x -q -m gpu --timeout 200 --timeout-method thread 2>&1 | tail -1
for v in 1 0 1 0 1 0; do
  PFSCDC_HASH_CU_EXCLUSIVE=$v timeout -k 10 300 python bench.py --config c3 --steps 4 --warmup 1 --no-cpu-baseline --no-e2e --no-chain-floor > gpurun_out/cx_$v.json 2>gpurun_out/cx_$v.err || { tail -3 gpurun_out/cx_$v.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/cx_$v.json').read().strip().splitlines()[-1]); k=d['kernel_ms']; print('c3 excl=$v', d['value'], d['ms_per_step'], round(k['hash'],2), round(k['hash_span'],2), d.get('index_digest'))"
done
for v in 1 0; do
  PFSCDC_HASH_CU_EXCLUSIVE=$v timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-chain-floor > gpurun_out/cx4_$v.json 2>gpurun_out/cx4_$v.err || { tail -3 gpurun_out/cx4_$v.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/cx4_$v.json').read().strip().splitlines()[-1]); k=d['kernel_ms']; print('c4 excl=$v', d['value'], d['ms_per_step'], round(k['hash'],2), d.get('index_digest'))"
done
