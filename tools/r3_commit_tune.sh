#!/bin/bash
# round 3: the c4 commit data plane at G=2 (in place) under the Ref.Id split knobs
mkdir -p gpurun_out/r3
run() {  # name env...
  name=$1; shift
  env "$@" timeout -k 10 400 python bench.py --config c4 --path commit --group 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r3/ct_$name.json 2> gpurun_out/r3/ct_$name.err || { tail -5 gpurun_out/r3/ct_$name.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r3/ct_$name.json').read().strip().splitlines()[-1]); print('$name', d['value'], d['ms_per_step'], d['kernel_ms'], d['commit_chunks_digest'])"
}
run base PFSCDC_NOTHING=0
run pct50 PFSCDC_REFID_LONG_PCT=50
run pct80 PFSCDC_REFID_LONG_PCT=80
run onestream PFSCDC_REFID_TWOSTREAM=0
run base2 PFSCDC_NOTHING=0
