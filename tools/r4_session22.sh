#!/bin/bash
# c4 one step at a time (each kernel alone) and c3, cut skipping off / on, alternating.
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/r4_ab_multi.sh r4cs6/c4 2 "PFSCDC_SCAN_CUTSKIP=0" "PFSCDC_SCAN_CUTSKIP=1" -- --config c4 --inflight 1 --steps 4 --warmup 2 --no-cpu-baseline --no-e2e --no-chain-floor &&
bash tools/r4_ab_multi.sh r4cs6/c3 1 "PFSCDC_SCAN_CUTSKIP=0" "PFSCDC_SCAN_CUTSKIP=1" -- --config c3 --steps 4 --warmup 2 --no-cpu-baseline --no-e2e --no-chain-floor
