#!/bin/bash
# c4 commit G=2 with the coalesced ChaCha20: the long chunk set's hash launches at two waves per
# SIMD (its union and its Ref.Id pass pick one by the chain-bound rule) vs the default.
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/r4_ab_env.sh r4ab_longwaves "PFSCDC_COMMIT_LONG_WAVES=0" "PFSCDC_COMMIT_LONG_WAVES=2 PFSCDC_COMMIT_LONG_CREATE_WAVES=2" 2 \
    --path commit --config c4 --group 2 --steps 3 --warmup 1 --no-cpu-baseline &&
bash tools/r4_ab_env.sh r4ab_longwaves2 "PFSCDC_COMMIT_LONG_WAVES=2" "PFSCDC_COMMIT_LONG_CREATE_WAVES=2" 1 \
    --path commit --config c4 --group 2 --steps 3 --warmup 1 --no-cpu-baseline
