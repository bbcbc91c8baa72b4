#!/bin/bash
# round 3: host-fed UnorderedWriter on 32 GiB of c4 with 8 / 16 / 32 GiB groups (one group
# writer): a group's GPU time is its two serial chains (~340 ms) whatever its size
mkdir -p gpurun_out/r3uwg
o=gpurun_out/r3uwg
for G in 8589934592 17179869184 34359738368; do
  timeout -k 10 500 python bench.py --path uw --config c4 --uw-bytes 34359738368 --uw-group $G --steps 2 --warmup 1 --no-cpu-baseline > $o/uw32_g$G.json 2> $o/uw32_g$G.err || { tail -5 $o/uw32_g$G.err; exit 1; }
  python -c "
import json; d=json.loads(open('$o/uw32_g$G.json').read().strip().splitlines()[-1])
print('uw32 group=$G', d['value'], d['ms_per_step'], {k: round(v,1) for k, v in d.get('stages_ms',{}).items()}, d.get('filesets_digest'))"
done
