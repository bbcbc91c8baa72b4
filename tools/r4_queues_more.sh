#!/bin/bash
# Hardware queues beyond c3: the host-fed writer with several group writers (each its own data
# ctx and index ctxs, plus the upload stream) and c4's commits in flight, at 32 queues.
set -o pipefail
cd "$(dirname "$0")/.."
o=gpurun_out/r4q
mkdir -p $o
uw() {  # name "ENV"
  env $2 timeout -k 10 300 python bench.py --path uw --config c4 --uw-bytes 34359738368 --steps 2 --warmup 1 > $o/$1.json 2> $o/$1.err || return 1
  python - $o/$1.json "$1 [$2]" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d["ms_per_step"], d["stages_ms"], d["commit_filesets_digest"])
PY
}
c4() {  # name "ENV" "args"
  env $2 timeout -k 10 300 python bench.py --config c4 --steps 6 --warmup 2 --no-cpu-baseline $3 > $o/$1.json 2> $o/$1.err || return 1
  python - $o/$1.json "$1 [$2] [$3]" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d["ms_per_step"], d["config"].get("steps_in_flight"), d["index_digest"])
PY
}
uw uw_w1_q32 "GPU_MAX_HW_QUEUES=32 PFSCDC_UW_WORKERS=1" &&
uw uw_w2_g16_q32 "GPU_MAX_HW_QUEUES=32 PFSCDC_UW_WORKERS=2 PFSCDC_UW_INFLIGHT=17179869184" &&
uw uw_w3_g8_q32 "GPU_MAX_HW_QUEUES=32 PFSCDC_UW_WORKERS=3 PFSCDC_UW_INFLIGHT=8589934592" &&
uw uw_w4_g8_q32 "GPU_MAX_HW_QUEUES=32 PFSCDC_UW_WORKERS=4 PFSCDC_UW_INFLIGHT=8589934592" &&
c4 c4_s2_q8 "GPU_MAX_HW_QUEUES=8" "" &&
c4 c4_s2_q16 "GPU_MAX_HW_QUEUES=16" ""
