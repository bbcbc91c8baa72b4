#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/r4_c3_sweep2.sh &&
bash tools/r4_queues_more.sh
