#!/bin/bash
# round 3: host-fed writer defaults (32 GiB groups, 40-arena pool): GPU fileset tests, then the
# 8 GiB and 32 GiB c4 Puts
mkdir -p gpurun_out/r3uwf
o=gpurun_out/r3uwf
timeout -k 10 300 python -u -m pytest tests/test_gpu_fileset.py tests/test_gpu_writer.py -x -q --timeout 200 --timeout-method thread > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
for B in 8589934592 34359738368; do
  timeout -k 10 500 python bench.py --path uw --config c4 --uw-bytes $B --steps 2 --warmup 1 --no-cpu-baseline > $o/uw_$B.json 2> $o/uw_$B.err || { tail -5 $o/uw_$B.err; exit 1; }
  python -c "
import json; d=json.loads(open('$o/uw_$B.json').read().strip().splitlines()[-1])
print('uw $B', d['value'], d['ms_per_step'], {k: round(v,1) for k, v in d.get('stages_ms',{}).items()}, d.get('filesets_digest'))"
done
