#!/bin/bash
# GPU suite + the commit data plane on c4 (two runs) and c5.
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_gpu.log 2>&1; tail -2 gpurun_out/t_gpu.log
for c in c4 c4 c5; do
  timeout -k 10 300 python bench.py --path commit --config $c --steps 3 --warmup 1 --no-e2e > gpurun_out/commit_$c.json 2>gpurun_out/commit_$c.err || { tail -3 gpurun_out/commit_$c.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/commit_$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'], d['kernel_ms'], d['commit_chunks_digest'], d['dataref_hashes_digest'], d.get('parity'))"
done
