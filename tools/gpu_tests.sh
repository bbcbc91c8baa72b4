#!/bin/bash
# GPU test run on the box: the selected test files (default: the whole GPU suite), one pytest
# process, each test under a thread timeout; output under gpurun_out/$NAME/.
#   bash tools/gpu_tests.sh NAME [pytest args...]
set -euo pipefail
cd "$(dirname "$0")/.."
NAME=${1:?name}; shift
O=gpurun_out/$NAME
mkdir -p $O
export TMPDIR=/tmp
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(tests -m gpu)
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread "${ARGS[@]}" \
  > $O/pytest.log 2>&1
tail -3 $O/pytest.log
