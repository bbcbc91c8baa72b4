#!/bin/bash
# (Historical: PFSCDC_HASH_PRIO, the hash launches' issue priority knob it sweeps, was removed in
# round 5 with the other rejected forms; the results are in profiles/r4/uw_sweep/.)
# Host-fed writer (32 GiB c4 Put): group writers in flight x group size x hash issue priority,
# after the grouped index close.  Each line: value, ms/step, stages, filesets digest.
set -o pipefail
cd "$(dirname "$0")/.."
o=gpurun_out/${1:-r4uw}
mkdir -p $o
run() {
  name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --path uw --config c4 --uw-bytes 34359738368 --steps 2 --warmup 1 > $o/$name.json 2> $o/$name.err || return 1
  python - $o/$name.json "$name $*" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d["ms_per_step"], d["stages_ms"], d["commit_filesets_digest"])
PY
}
run w1_g32 PFSCDC_UW_WORKERS=1 &&
run w2_g16 PFSCDC_UW_WORKERS=2 PFSCDC_UW_INFLIGHT=17179869184 &&
run w2_g8 PFSCDC_UW_WORKERS=2 PFSCDC_UW_INFLIGHT=8589934592 &&
run w3_g8 PFSCDC_UW_WORKERS=3 PFSCDC_UW_INFLIGHT=8589934592 &&
run w2_g16_prio PFSCDC_UW_WORKERS=2 PFSCDC_UW_INFLIGHT=17179869184 PFSCDC_HASH_PRIO=1 &&
run w3_g8_prio PFSCDC_UW_WORKERS=3 PFSCDC_UW_INFLIGHT=8589934592 PFSCDC_HASH_PRIO=1 &&
run w1_g32_again PFSCDC_UW_WORKERS=1
