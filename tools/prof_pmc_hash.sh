# PMC passes for the hash kernel (bench-shaped workload, 4096 x 4 MiB)
mkdir -p gpurun_out && export TMPDIR=/tmp
P="python tools/prof_driver.py 1 4096"
run() { timeout -k 10 200 rocprofv3 --kernel-include-regex "$1" --pmc $2 -d gpurun_out/$3 -o p --output-format csv -- $P > gpurun_out/$3.log 2>&1; }
run blake2b "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS" hash_sq && \
run blake2b "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU" hash_lds
echo rc=$?
