#!/bin/bash
# The c2 line at 8 vs 32 hardware queues (the c2 default is now 32, for the literal leg's
# twelve batches in flight), then the full default line once (the literal leg's new
# many_in_flight figure).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r4s12
bash tools/r4_ab_env.sh r4ab_q "GPU_MAX_HW_QUEUES=8" "GPU_MAX_HW_QUEUES=32" 2 &&
timeout -k 10 400 python bench.py > gpurun_out/r4s12/bench.json 2> gpurun_out/r4s12/bench.err &&
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r4s12/bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["config"]["gpu_max_hw_queues"], d["configs1_literal"], d["roofline"]["frac"])
PY
