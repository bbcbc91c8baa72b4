#!/bin/bash
# round 3: host-fed UnorderedWriter on 32 GiB of c4 (4 groups of 8 GiB) with 1/2/3 group
# writers in flight, now that bench.py gives the process 8 hardware queues
mkdir -p gpurun_out/r3uw
o=gpurun_out/r3uw
for W in 1 2 3; do
  PFSCDC_TRACE=0 timeout -k 10 500 python bench.py --path uw --config c4 --uw-bytes 34359738368 --uw-workers $W --steps 2 --warmup 1 --no-cpu-baseline > $o/uw32_w$W.json 2> $o/uw32_w$W.err || { tail -5 $o/uw32_w$W.err; exit 1; }
  python -c "
import json; d=json.loads(open('$o/uw32_w$W.json').read().strip().splitlines()[-1])
print('uw32 W=$W', d['value'], d['ms_per_step'], {k: round(v,1) for k, v in d.get('stages_ms',{}).items()}, d.get('filesets_digest'))"
done
