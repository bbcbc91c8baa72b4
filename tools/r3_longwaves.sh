#!/bin/bash
# round 3: the two-set commit's long set at one wave per SIMD (its chains at the lone-wave
# rate, PFSCDC_COMMIT_LONG_WAVES=1) against its own choice; c4 G=2 in place, alternating
mkdir -p gpurun_out/r3lw
o=gpurun_out/r3lw
run() {  # name long_waves pct
  PFSCDC_COMMIT_LONG_WAVES=$2 PFSCDC_COMMIT_LONG_PCT=$3 timeout -k 10 400 python bench.py --config c4 --path commit --group 2 --steps 3 --warmup 1 --no-cpu-baseline > $o/$1.json 2> $o/$1.err || { tail -5 $o/$1.err; exit 1; }
  python -c "
import json; d=json.loads(open('$o/$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('$1', d['value'], d['ms_per_step'], round(k['scan'],1), round(k['create_content_hash'],1), round(k['create'],1), d['commit_chunks_digest'], d['dataref_hashes_digest'])"
}
for r in 1 2; do
run own30_$r 0 30
run lw1_30_$r 1 30
done
run lw1_20 1 20
run lw1_40 1 40
run lw1_50 1 50
