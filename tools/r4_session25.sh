#!/bin/bash
# What the rank order costs, by footprint: the c2 line at 8 batches per step (32 GiB, 8,192
# files) and at 32 (128 GiB), cut skipping off / rank order alone, alternating.
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/r4_ab_multi.sh r4ord/g8 3 "PFSCDC_SCAN_CUTSKIP=0" "PFSCDC_SCAN_CUTSKIP=3" -- --group 8 --steps 20 --warmup 4 --no-cpu-baseline --no-e2e --no-literal --no-pipelined --no-chain-floor &&
bash tools/r4_ab_multi.sh r4ord/g32 2 "PFSCDC_SCAN_CUTSKIP=0" "PFSCDC_SCAN_CUTSKIP=3"
