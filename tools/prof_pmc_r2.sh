#!/bin/bash
# PMC passes for the hash and scan kernels on one c2-sized launch (32768 x 4 MiB = 128 GiB),
# one counter group per pass (each pass its own limit), then a readable summary.
mkdir -p gpurun_out && export TMPDIR=/tmp
P="python tools/prof_driver.py 1 32768"
run() { timeout -s KILL 200 rocprofv3 --kernel-include-regex "$1" --pmc $2 -d gpurun_out/$3 -o p --output-format csv -- $P > gpurun_out/$3.log 2>&1; }
run blake2b "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS" hash_sq && \
run blake2b "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU" hash_lds && \
run cdc_scan "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS" scan_sq && \
run cdc_scan "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU" scan_lds
rc=$?
python tools/pmc_summary.py gpurun_out/hash_sq gpurun_out/hash_lds gpurun_out/scan_sq gpurun_out/scan_lds > gpurun_out/pmc_r2.txt 2>&1
cat gpurun_out/pmc_r2.txt
exit $rc
