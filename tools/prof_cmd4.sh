mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 120 ./tools/ubench > gpurun_out/ubench.txt 2>&1 && \
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1 ; \
timeout -k 10 200 rocprofv3 --kernel-include-regex cdc_scan --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/pmc1 -o p --output-format csv -- python tools/prof_driver.py 2 > gpurun_out/pmc1.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-include-regex cdc_scan --pmc FETCH_SIZE -d gpurun_out/pmc2 -o p --output-format csv -- python tools/prof_driver.py 2 > gpurun_out/pmc2.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-include-regex cdc_scan --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc3 -o p --output-format csv -- python tools/prof_driver.py 2 > gpurun_out/pmc3.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-include-regex blake2b --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/pmc4 -o p --output-format csv -- python tools/prof_driver.py 1 > gpurun_out/pmc4.log 2>&1
echo rc=$?
