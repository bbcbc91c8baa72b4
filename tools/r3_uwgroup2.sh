#!/bin/bash
# round 3: 16 / 32 GiB groups with an arena pool that holds a whole step (PFSCDC_UW_ARENA_POOL)
mkdir -p gpurun_out/r3uwg2
o=gpurun_out/r3uwg2
for G in 17179869184 34359738368; do
  PFSCDC_UW_ARENA_POOL=40 timeout -k 10 500 python bench.py --path uw --config c4 --uw-bytes 34359738368 --uw-group $G --steps 2 --warmup 1 --no-cpu-baseline > $o/uw32_g$G.json 2> $o/uw32_g$G.err || { tail -5 $o/uw32_g$G.err; exit 1; }
  python -c "
import json; d=json.loads(open('$o/uw32_g$G.json').read().strip().splitlines()[-1])
print('uw32 pool40 group=$G', d['value'], d['ms_per_step'], {k: round(v,1) for k, v in d.get('stages_ms',{}).items()}, d.get('filesets_digest'))"
done
PFSCDC_UW_ARENA_POOL=40 timeout -k 10 500 python bench.py --path uw --config c4 --uw-bytes 8589934592 --uw-group 8589934592 --steps 3 --warmup 1 --no-cpu-baseline > $o/uw8.json 2> $o/uw8.err || { tail -5 $o/uw8.err; exit 1; }
python -c "
import json; d=json.loads(open('$o/uw8.json').read().strip().splitlines()[-1])
print('uw8 pool40', d['value'], d['ms_per_step'], {k: round(v,1) for k, v in d.get('stages_ms',{}).items()})"
