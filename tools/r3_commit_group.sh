#!/bin/bash
# round 3: commit data plane and the every-BLAKE2b line with G commits per step (one GPU)
mkdir -p gpurun_out/r3
for G in 2 3; do
  for mode in hashes commit; do
    extra=""; [ $mode = hashes ] && extra="--no-create"
    timeout -k 10 400 python bench.py --config c4 --path commit $extra --group $G --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r3/c4_${mode}_g$G.json 2> gpurun_out/r3/c4_${mode}_g$G.err || { tail -5 gpurun_out/r3/c4_${mode}_g$G.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/r3/c4_${mode}_g$G.json').read().strip().splitlines()[-1]); print('$mode G=$G', d['value'], d['ms_per_step'], d['kernel_ms'], d['commit_chunks_digest'], d['dataref_hashes_digest'])"
  done
done
