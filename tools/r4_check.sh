#!/bin/bash
# The driver's sequence on the tree after a host-side change: the GPU suite, smoke(), the
# default line.
set -o pipefail
cd "$(dirname "$0")/.."
o=gpurun_out/r4chk
mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $o/pytest_gpu.log 2>&1 && tail -1 $o/pytest_gpu.log &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 && tail -1 $o/smoke.log &&
timeout -k 10 400 python bench.py > $o/bench.json 2> $o/bench.err &&
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r4chk/bench.json").read().strip().splitlines()[-1])
k = d["kernel_ms"]
print(d["value"], d["ms_per_step"], round(k["scan"], 2), round(k["hash"], 2), round(k["scan_mhz"]), round(k["hash_mhz"]), d["roofline"]["frac"], d["roofline_cdc"]["rolled_fraction"], d["parity"]["gpu_equals_cpu_oracle"], d["two_in_flight"]["value"])
PY
