#!/bin/bash
# Same-box A/B of environment knobs on the c2 line (one step in flight, no side legs).
# usage: bash tools/ab_env.sh <reps> "<ENV A>" "<ENV B>" ...   (each arg: space-separated K=V, or "-")
mkdir -p gpurun_out/abenv
R=$1; shift
B="--steps 6 --warmup 2 --no-e2e --no-cpu-baseline --no-literal --no-pipelined --no-chain-floor"
for i in $(seq 1 $R); do
  k=0
  for e in "$@"; do
    k=$((k+1))
    envs=""; [ "$e" != "-" ] && envs="$e"
    env $envs timeout -k 10 200 python bench.py $B > gpurun_out/abenv/v${k}_$i.json 2>gpurun_out/abenv/v${k}_$i.err || exit 1
    python -c "
import json
d=json.load(open('gpurun_out/abenv/v${k}_$i.json')); k=d['kernel_ms']; print('v$k', '$e', d['value'], round(k['scan'],2), round(k['hash'],2), flush=True)"
  done
done
