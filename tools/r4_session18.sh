#!/bin/bash
# Cut skipping with the plan kernels' atomics aggregated per block: the cut-skip parity cases,
# then a same-box four-arm A/B of the c2 line: off, full, rank order + reports without
# skipping, rank order alone.
set -o pipefail
cd "$(dirname "$0")/.."
o=gpurun_out/r4cs2
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "skip" --timeout 200 --timeout-method thread > $o/pytest_skip.log 2>&1 && tail -1 $o/pytest_skip.log &&
bash tools/r4_ab_multi.sh r4ab_cs4 2 "PFSCDC_SCAN_CUTSKIP=0" "PFSCDC_SCAN_CUTSKIP=1" "PFSCDC_SCAN_CUTSKIP=2" "PFSCDC_SCAN_CUTSKIP=3"
