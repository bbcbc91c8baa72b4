# PMC passes (one counter group per pass, kernel-trace off) for the scan and hash kernels.
mkdir -p gpurun_out && export TMPDIR=/tmp
P="python tools/prof_driver.py 2"
run() { timeout -k 10 200 rocprofv3 --kernel-include-regex "$1" --pmc $2 -d gpurun_out/$3 -o p --output-format csv -- $P > gpurun_out/$3.log 2>&1; }
run cdc_scan "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS" scan_sq && \
run cdc_scan "FETCH_SIZE" scan_fetch && \
run cdc_scan "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD" scan_lds && \
run blake2b "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS" hash_sq && \
run blake2b "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES" hash_misc
echo rc=$?
