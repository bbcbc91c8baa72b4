#!/bin/bash
# Round 6: the host sanitizer runs (ASan/LSan/UBSan, then TSan) over the C drivers, the
# unordered writer driver now with a device group, then a soak of the device group's
# randomised GPU tests.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/${1:-r6san}
mkdir -p $o
bash tools/host_sanitize.sh run $o/asan > $o/asan.txt 2>&1; echo "asan rc=$?"; tail -3 $o/asan.txt
bash tools/host_sanitize.sh run-tsan $o/tsan > $o/tsan.txt 2>&1; echo "tsan rc=$?"; tail -3 $o/tsan.txt
PFS_FUZZ_CASES=25 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_group.py -k "host_equals" > $o/soak_group.log 2>&1; echo "soak rc=$?"; tail -2 $o/soak_group.log
