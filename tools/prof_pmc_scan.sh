# PMC passes for the scan kernel (bench-shaped workload, 8192 x 4 MiB)
mkdir -p gpurun_out && export TMPDIR=/tmp
P="python tools/prof_driver.py 1 8192"
run() { timeout -k 10 200 rocprofv3 --kernel-include-regex "$1" --pmc $2 -d gpurun_out/$3 -o p --output-format csv -- $P > gpurun_out/$3.log 2>&1; }
run cdc_scan "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS" scan_sq && \
run cdc_scan "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES" scan_misc && \
run cdc_scan "SQ_INSTS_SMEM SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE" scan_more
echo rc=$?
