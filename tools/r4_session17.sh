#!/bin/bash
# Cut skipping past settled first cuts (ScanPlan): the parity file first, then the same-box
# A/B of the c2 line (PFSCDC_SCAN_CUTSKIP=0 / 1), then the whole GPU suite.
set -o pipefail
cd "$(dirname "$0")/.."
o=gpurun_out/r4cs
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > $o/pytest_parity.log 2>&1 && tail -1 $o/pytest_parity.log &&
bash tools/r4_ab_env.sh r4ab_cs "PFSCDC_SCAN_CUTSKIP=0" "PFSCDC_SCAN_CUTSKIP=1" 3 &&
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $o/pytest_gpu.log 2>&1 && tail -1 $o/pytest_gpu.log
