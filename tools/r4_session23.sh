#!/bin/bash
# The serial tails batched (scan compaction, segment compaction, LPT order: kSerialK items per
# thread and pass): the GPU suite, then a same-box A/B against the library before the change.
set -o pipefail
cd "$(dirname "$0")/.."
o=gpurun_out/r4ser
mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $o/pytest_gpu.log 2>&1 && tail -1 $o/pytest_gpu.log &&
bash tools/r4_ab_multi.sh r4ser/c2 3 "PFSCDC_LIB=pfs_amd/ab/libpfscdc_base.so" "PFSCDC_X=1"
