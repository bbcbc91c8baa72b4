#!/bin/bash
# round 3: the long set's union at one wave per SIMD, its chunk.Create at its own waves
mkdir -p gpurun_out/r3lw2
o=gpurun_out/r3lw2
run() {  # name union_waves create_waves pct
  PFSCDC_COMMIT_LONG_WAVES=$2 PFSCDC_COMMIT_LONG_CREATE_WAVES=$3 PFSCDC_COMMIT_LONG_PCT=$4 timeout -k 10 400 python bench.py --config c4 --path commit --group 2 --steps 3 --warmup 1 --no-cpu-baseline > $o/$1.json 2> $o/$1.err || { tail -5 $o/$1.err; exit 1; }
  python -c "
import json; d=json.loads(open('$o/$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('$1', d['value'], d['ms_per_step'], round(k['scan'],1), round(k['create_content_hash'],1), round(k['create'],1), d['commit_chunks_digest'], d['dataref_hashes_digest'])"
}
for r in 1 2; do
run own30_$r 0 0 30
run u1_30_$r 1 0 30
done
run u1_40 1 0 40
run u1_50 1 0 50
