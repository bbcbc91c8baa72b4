#!/bin/bash
# Round 6: hash waves per SIMD on the default line (PFSCDC_HASH_WAVES), same box, alternating.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/${1:-r6hw}
mkdir -p $o
B="--no-cpu-baseline --no-e2e --no-literal --no-pipelined --no-chain-floor --steps 10 --warmup 3"
run() { name=$1; shift; env "$@" timeout -k 10 300 python bench.py $B > $o/$name.json 2> $o/$name.err && \
  python -c "import json; d=json.load(open('$o/$name.json')); k=d['kernel_ms']; print('$name', d['value'], d['ms_per_step'], round(k['hash'],2), round(k['hash_mhz']), round(k['scan'],2), round(k['scan_mhz']), d['config'].get('index_digest', d.get('index_digest')))"; }
run w2a PFSCDC_HASH_WAVES=0 && run w1a PFSCDC_HASH_WAVES=1 && run w3a PFSCDC_HASH_WAVES=3 &&
run w2b PFSCDC_HASH_WAVES=0 && run w1b PFSCDC_HASH_WAVES=1 && run w3b PFSCDC_HASH_WAVES=3
