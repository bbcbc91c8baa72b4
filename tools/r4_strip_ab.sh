#!/bin/bash
# 8 KiB strips (512 KiB work units: half as many unit starts, each in a file of its own in
# the rank order) against the 4 KiB default, cut skipping on; then the parity file on the
# 8 KiB build (pfs_amd/ab/libpfscdc_s8k.so: -DPFS_SCAN_STRIP=8192).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r4s8k
bash tools/r4_ab_multi.sh r4s8k 3 "PFSCDC_X=0" "PFSCDC_LIB=pfs_amd/ab/libpfscdc_s8k.so" &&
PFSCDC_LIB=pfs_amd/ab/libpfscdc_s8k.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r4s8k/pytest_parity.log 2>&1; tail -1 gpurun_out/r4s8k/pytest_parity.log
