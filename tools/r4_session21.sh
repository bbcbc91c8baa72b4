#!/bin/bash
# Cut skipping past every settled cut (per-file rank slots, the selection replayed over them):
# the skip parity cases, then same-box A/Bs of the c2 line, c4 and the c4 commit data plane,
# then the whole GPU suite.
set -o pipefail
cd "$(dirname "$0")/.."
o=gpurun_out/r4cs5
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "skip" --timeout 200 --timeout-method thread > $o/pytest_skip.log 2>&1 && tail -1 $o/pytest_skip.log &&
bash tools/r4_ab_multi.sh r4cs5/c2 2 "PFSCDC_SCAN_CUTSKIP=0" "PFSCDC_SCAN_CUTSKIP=1" "PFSCDC_SCAN_CUTSKIP=2" &&
bash tools/r4_ab_multi.sh r4cs5/c4 1 "PFSCDC_SCAN_CUTSKIP=0" "PFSCDC_SCAN_CUTSKIP=1" -- --config c4 --steps 4 --warmup 2 --no-cpu-baseline --no-e2e --no-chain-floor &&
bash tools/r4_ab_multi.sh r4cs5/commit 1 "PFSCDC_SCAN_CUTSKIP=0" "PFSCDC_SCAN_CUTSKIP=1" -- --path commit --config c4 --group 2 --steps 3 --warmup 1 --no-cpu-baseline &&
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $o/pytest_gpu.log 2>&1 && tail -1 $o/pytest_gpu.log
