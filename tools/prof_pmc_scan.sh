mkdir -p gpurun_out && export TMPDIR=/tmp
P="python tools/prof_driver.py 2"
run() { timeout -k 10 200 rocprofv3 --kernel-include-regex "$1" --pmc $2 -d gpurun_out/$3 -o p --output-format csv -- $P > gpurun_out/$3.log 2>&1; }
run cdc_scan "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS" scan_sq && \
run cdc_scan "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" scan_misc && \
run cdc_scan "FETCH_SIZE" scan_fetch
echo rc=$?
