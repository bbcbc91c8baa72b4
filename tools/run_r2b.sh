#!/bin/bash
# Round-2 (second session) artifacts: GPU tests, smoke, the PMC pass of the bench workload
# (FETCH_SIZE + SQ_INSTS_VALU per launch -> traffic json), the default bench line with it, and
# a kernel-trace --stats pass of the bench's 128 GiB steps.  Every GPU step has its own limit.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out && export TMPDIR=/tmp
B="--no-cpu-baseline --no-e2e --no-literal --no-pipelined --no-chain-floor"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-include-regex "blake2b|cdc_scan" --pmc FETCH_SIZE SQ_INSTS_VALU -d gpurun_out/pmc_fetch -o p --output-format csv -- python bench.py --steps 2 --warmup 1 $B > gpurun_out/pmc_fetch.log 2>&1 && \
python tools/traffic.py gpurun_out/pmc_fetch gpurun_out/traffic.json > gpurun_out/traffic.log 2>&1 && \
timeout -k 10 400 python bench.py --traffic-json gpurun_out/traffic.json > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats -o run --output-format csv -- python bench.py --steps 20 --warmup 5 $B > gpurun_out/prof_stats.log 2>&1
rc=$?
echo rc=$rc
exit $rc
