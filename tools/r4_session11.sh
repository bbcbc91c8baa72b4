#!/bin/bash
# The c3 line with its new defaults (12 streams, 32 queues, scan grid 64), three runs; and the
# GPU tests that the bench/default changes touch.
set -o pipefail
cd "$(dirname "$0")/.."
o=gpurun_out/r4s11
mkdir -p $o
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --config c3 --steps 12 --warmup 3 --no-cpu-baseline > $o/c3_$i.json 2> $o/c3_$i.err || exit 1
  python - $o/c3_$i.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernel_ms"]
print(sys.argv[1].split("/")[-1], d["value"], d["ms_per_step"], d["config"]["steps_in_flight"], d["config"]["gpu_max_hw_queues"], d["config"].get("scan_grid"), round(k["scan"], 2), round(k["hash"], 1), d.get("one_step_alone", {}).get("value"), d["index_digest"])
PY
done
