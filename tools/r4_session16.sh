#!/bin/bash
# The driver's sequence on the current tree first (GPU suite, smoke, default line), then the
# four-rank rehearsal, the c2 queue A/B and the scan-waves A/Bs.
set -o pipefail
cd "$(dirname "$0")/.."
o=gpurun_out/r4dl
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $o/pytest_gpu.log 2>&1 && tail -1 $o/pytest_gpu.log &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 && tail -1 $o/smoke.log &&
timeout -k 10 400 python bench.py > $o/bench.json 2> $o/bench.err &&
python - <<'PY' &&
import json
d = json.loads(open("gpurun_out/r4dl/bench.json").read().strip().splitlines()[-1])
k = d["kernel_ms"]
print(d["value"], d["ms_per_step"], round(k["scan"], 2), round(k["hash"], 2), round(k["scan_mhz"]), round(k["hash_mhz"]), d["roofline"]["frac"], d["config"]["gpu_max_hw_queues"], d["parity"], d["configs1_literal"].get("many_in_flight"), d["cpu_baseline"]["value"])
PY
bash tools/rehearse_r4_n4.sh &&
bash tools/r4_ab_env.sh r4ab_q "GPU_MAX_HW_QUEUES=8" "GPU_MAX_HW_QUEUES=32" 2 &&
bash tools/r4_session14.sh
