#!/bin/bash
# Round 4, second GPU session: the pair-form scan after the in-flight register fix (parity,
# then a same-box A/B whose digests must now agree), and the host-fed writer with the grouped
# index close (fileset GPU tests, then a 32 GiB c4 Put A/B).
set -o pipefail
cd "$(dirname "$0")/.."
o=gpurun_out/r4s2
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fileset.py tests/test_gpu_distributed.py -x -q --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 && tail -1 $o/pytest.log &&
bash tools/r4_ab_env.sh r4ab_pair2 "PFSCDC_SCAN_PAIR=0" "PFSCDC_SCAN_PAIR=1" 3 &&
bash tools/r4_ab_env.sh r4ab_uwidx "PFSCDC_UW_INDEX_GROUPED=0" "PFSCDC_UW_INDEX_GROUPED=1" 2 \
    --path uw --config c4 --uw-bytes 34359738368 --steps 2 --warmup 1 &&
o2=gpurun_out/r4s2
PFSCDC_TRACE=1 timeout -k 10 300 python bench.py --path commit --config c4 --group 2 --steps 3 --warmup 1 --no-cpu-baseline > $o2/commit_g2_trace.json 2> $o2/commit_g2_trace.err && grep "two sets" $o2/commit_g2_trace.err | tail -3 && python -c "
import json; d=json.loads(open('$o2/commit_g2_trace.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernel_ms'])"
