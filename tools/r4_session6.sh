#!/bin/bash
# Coalesced ChaCha20 pass: parity (Ref.Id, commit, in place), then same-box A/Bs on the c4 G=2
# commit data plane and the 32 GiB host-fed Put; digests must not change.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r4s6
timeout -k 10 400 python -u -m pytest tests/test_gpu_refid.py tests/test_gpu_commit.py tests/test_gpu_writer.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4s6/pytest.log 2>&1 && tail -1 gpurun_out/r4s6/pytest.log &&
bash tools/r4_ab_env.sh r4ab_chacha "PFSCDC_CHACHA_COALESCED=0" "PFSCDC_CHACHA_COALESCED=1" 3 \
    --path commit --config c4 --group 2 --steps 3 --warmup 1 --no-cpu-baseline &&
bash tools/r4_ab_env.sh r4ab_chacha_uw "PFSCDC_CHACHA_COALESCED=0" "PFSCDC_CHACHA_COALESCED=1" 1 \
    --path uw --config c4 --uw-bytes 34359738368 --steps 2 --warmup 1
