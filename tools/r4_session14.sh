#!/bin/bash
# Scan waves per CU (compile-time PFS_SCAN_WAVES): the default 12 (3 per SIMD, LDS full) against
# 8 and 4 (fewer waves, less power, maybe a higher clock), same box, alternating; digests equal.
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/r4_ab_env.sh r4ab_w8 "PFSCDC_LIB=pfs_amd/libpfscdc.so" "PFSCDC_LIB=pfs_amd/ab/libpfscdc_w8.so" 2 &&
bash tools/r4_ab_env.sh r4ab_w4 "PFSCDC_LIB=pfs_amd/libpfscdc.so" "PFSCDC_LIB=pfs_amd/ab/libpfscdc_w4.so" 1 &&
bash tools/r4_ab_env.sh r4ab_w8a14 "PFSCDC_LIB=pfs_amd/libpfscdc.so" "PFSCDC_LIB=pfs_amd/ab/libpfscdc_w8a14.so" 1
