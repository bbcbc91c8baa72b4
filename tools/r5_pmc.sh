#!/bin/bash
# Final-tree PMC of the two dominant kernels on the default workload (128 GiB steps), one
# rocprofv3 --pmc pass per counter group (8 SQ counters; then the LDS/busy group), and a
# per-kernel, per-dispatch summary (tools/pmc_per_kernel.py).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/${1:-r5pmc}
mkdir -p $o
B="--no-cpu-baseline --no-e2e --no-literal --no-pipelined --no-chain-floor --steps 2 --warmup 1"
timeout -s KILL 240 rocprofv3 --kernel-include-regex "blake2b|cdc_scan" --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d $o/sq -o p --output-format csv -- python3 bench.py $B > $o/sq.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --kernel-include-regex "blake2b|cdc_scan" --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d $o/lds -o p --output-format csv -- python3 bench.py $B > $o/lds.log 2>&1 &&
python tools/pmc_per_kernel.py $o/sq $o/lds > $o/pmc_summary.txt && cat $o/pmc_summary.txt
