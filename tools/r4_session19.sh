#!/bin/bash
# Cut skipping on the other configurations: the GPU suite and smoke() on the tree, then
# same-box A/Bs (PFSCDC_SCAN_CUTSKIP=0 / 1) of c3, c4, the c4 commit data plane and the
# default bench line.
set -o pipefail
cd "$(dirname "$0")/.."
o=gpurun_out/r4cs3
mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $o/pytest_gpu.log 2>&1 && tail -1 $o/pytest_gpu.log &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 && tail -1 $o/smoke.log &&
bash tools/r4_ab_multi.sh r4cs3/c4 1 "PFSCDC_SCAN_CUTSKIP=0" "PFSCDC_SCAN_CUTSKIP=1" -- --config c4 --steps 4 --warmup 2 --no-cpu-baseline --no-e2e --no-chain-floor &&
bash tools/r4_ab_multi.sh r4cs3/commit 1 "PFSCDC_SCAN_CUTSKIP=0" "PFSCDC_SCAN_CUTSKIP=1" -- --path commit --config c4 --group 2 --steps 3 --warmup 1 --no-cpu-baseline &&
bash tools/r4_ab_multi.sh r4cs3/c3 1 "PFSCDC_SCAN_CUTSKIP=0" "PFSCDC_SCAN_CUTSKIP=1" -- --config c3 --steps 4 --warmup 2 --no-cpu-baseline --no-e2e --no-chain-floor &&
bash tools/r4_ab_multi.sh r4cs3/default 2 "PFSCDC_SCAN_CUTSKIP=0" "PFSCDC_SCAN_CUTSKIP=1" -- --no-cpu-baseline
