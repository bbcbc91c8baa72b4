#!/bin/bash
# c4 commit: the two-stream Ref.Id pass's long subset (cost model, fixed percentages, one stream)
for v in model 65 model 0; do
  E="PFSCDC_REFID_LONG_PCT=$v"; [ $v = model ] && E="PFSCDC_REFID_LONG_PCT=0"; [ $v = 0 ] && E="PFSCDC_REFID_TWOSTREAM=0"
  env $E timeout -k 10 300 python bench.py --path commit --config c4 --steps 3 --warmup 1 --no-e2e --no-cpu-baseline > gpurun_out/lp_$v.json 2>gpurun_out/lp_$v.err || { tail -3 gpurun_out/lp_$v.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/lp_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['kernel_ms']['create_content_hash'], d['kernel_ms']['create_ref_id'], d['commit_chunks_digest'])"
done
