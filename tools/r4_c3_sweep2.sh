#!/bin/bash
# configs[2]: streams in flight x hardware queues (one HIP stream per context; streams beyond
# the process's queues share one and serialize).  Digest must not change.
set -o pipefail
cd "$(dirname "$0")/.."
o=gpurun_out/${1:-r4c3b}
mkdir -p $o
run() {  # name "ENV=..." "bench args"
  name=$1
  env $2 timeout -k 10 300 python bench.py --config c3 --steps 12 --warmup 3 --no-cpu-baseline $3 > $o/$name.json 2> $o/$name.err || return 1
  python - $o/$name.json "$name [$2] [$3]" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernel_ms"]
print(sys.argv[2], d["value"], d["ms_per_step"], "S", d["config"].get("steps_in_flight"), "q", d["config"].get("gpu_max_hw_queues"), "scan", round(k["scan"], 2), "hash", round(k["hash"], 1), d.get("one_step_alone", {}).get("value"), d["index_digest"])
PY
}
run s4_q16 "GPU_MAX_HW_QUEUES=16" "--inflight 4" &&
run s8_q16 "GPU_MAX_HW_QUEUES=16" "--inflight 8" &&
run s8_q24 "GPU_MAX_HW_QUEUES=24" "--inflight 8" &&
run s10_q24 "GPU_MAX_HW_QUEUES=24" "--inflight 10" &&
run s12_q32 "GPU_MAX_HW_QUEUES=32" "--inflight 12" &&
run s12_q32_g64 "GPU_MAX_HW_QUEUES=32 PFSCDC_SCAN_GRID=64" "--inflight 12" &&
run s16_q32 "GPU_MAX_HW_QUEUES=32" "--inflight 16"
