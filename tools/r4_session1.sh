#!/bin/bash
# Round 4, first GPU session: the driver's sequence and the N=2 self-launch (r4_verify.sh),
# then same-box A/Bs of the pair-form scan and of the graded fair share.
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/r4_verify.sh r4v1 &&
bash tools/r4_ab_env.sh r4ab_pair "PFSCDC_SCAN_PAIR=0" "PFSCDC_SCAN_PAIR=1" 3 &&
bash tools/r4_ab_env.sh r4ab_fair "PFSCDC_HASH_FAIR_GRADED=0" "PFSCDC_HASH_FAIR_GRADED=1 PFSCDC_HASH_FAIR_EVERY=512" 3
