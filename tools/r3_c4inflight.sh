#!/bin/bash
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3c4_parity.log 2>&1 || { tail -30 gpurun_out/r3c4_parity.log; exit 1; }; tail -1 gpurun_out/r3c4_parity.log
# round 3: c4 / c5 with one and two commits in flight (two contexts), 8 hardware queues
mkdir -p gpurun_out/r3c4
o=gpurun_out/r3c4
for cfg in c4 c5; do
for S in 1 2; do
  timeout -k 10 400 python bench.py --config $cfg --inflight $S --steps 4 --warmup 2 --no-cpu-baseline --no-e2e --no-literal --no-pipelined --no-chain-floor > $o/${cfg}_s$S.json 2> $o/${cfg}_s$S.err || { tail -5 $o/${cfg}_s$S.err; exit 1; }
  python -c "
import json; d=json.loads(open('$o/${cfg}_s$S.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('$cfg S=$S', d['value'], d['ms_per_step'], round(k['scan'],1), round(k['hash'],1), d.get('index_digest'), d.get('single_commit',{}).get('value'))"
done
done
