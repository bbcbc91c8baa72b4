#!/bin/bash
# c2 line at several launch-group sizes (batches of 1024 x 4 MiB per step).
N="--steps 6 --warmup 2 --no-e2e --no-cpu-baseline --no-literal --no-pipelined --no-chain-floor"
for g in "$@"; do
  timeout -k 10 300 python bench.py $N --group $g > gpurun_out/g$g.json 2>gpurun_out/g$g.err || { tail -3 gpurun_out/g$g.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/g$g.json').read().strip().splitlines()[-1]); k=d['kernel_ms']; print($g, d['value'], d['ms_per_step'], round(k['scan'],2), round(k['hash'],2), d['segments_per_step'], flush=True)"
done
