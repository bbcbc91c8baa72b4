#!/bin/bash
# Where the c4 G=2 commit step's issue slots go: a kernel trace (overlap, per-launch spans) and
# one PMC pass of SQ_INSTS_VALU per launch (the VALU work of one step against what the SIMDs
# could issue in the step's time).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/r4s7
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace -d $o/kt -o run --output-format csv -- python3 bench.py --path commit --config c4 --group 2 --steps 2 --warmup 1 --no-cpu-baseline > $o/kt.json 2> $o/kt.err &&
timeout -s KILL 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -d $o/pmc -o p --output-format csv -- python3 bench.py --path commit --config c4 --group 2 --steps 1 --warmup 1 --no-cpu-baseline > $o/pmc.json 2> $o/pmc.err &&
ls $o/kt $o/pmc
