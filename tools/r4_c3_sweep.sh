#!/bin/bash
# configs[2] (one 10 GiB stream per step, several in flight): the scan's workgroups capped so a
# step's scan never waits for CUs held by the other streams' chain-bound hash launches, more
# streams in flight, more hardware queues.  Digest must not change.
set -o pipefail
cd "$(dirname "$0")/.."
o=gpurun_out/${1:-r4c3}
mkdir -p $o
run() {  # name "ENV=..." "bench args"
  name=$1
  env $2 timeout -k 10 300 python bench.py --config c3 --steps 8 --warmup 2 --no-cpu-baseline $3 > $o/$name.json 2> $o/$name.err || return 1
  python - $o/$name.json "$name [$2] [$3]" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernel_ms"]
print(sys.argv[2], d["value"], d["ms_per_step"], "S", d["config"].get("steps_in_flight"), "scan", round(k["scan"], 2), "hash", round(k["hash"], 1), d.get("one_step_alone", {}).get("value"), d["index_digest"])
PY
}
run base "PFSCDC_SCAN_GRID=0" "" &&
run grid128 "PFSCDC_SCAN_GRID=128" "" &&
run grid64 "PFSCDC_SCAN_GRID=64" "" &&
run grid64_s6_q12 "PFSCDC_SCAN_GRID=64 GPU_MAX_HW_QUEUES=12" "--inflight 6" &&
run grid32_s8_q16 "PFSCDC_SCAN_GRID=32 GPU_MAX_HW_QUEUES=16" "--inflight 8" &&
run s8_q16 "GPU_MAX_HW_QUEUES=16" "--inflight 8"
