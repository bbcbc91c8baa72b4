#!/bin/bash
# Round-2 artifacts for the current tree: GPU tests, smoke, PMC pass (traffic json), the
# default bench line, a kernel-trace --stats pass, c3/c4 lines and a c2 N=2 rehearsal
# (two ranks on the one GPU, gloo).  Every GPU step has its own time limit.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out && export TMPDIR=/tmp
B="--no-cpu-baseline --no-e2e --no-literal --no-pipelined --no-chain-floor"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-include-regex "blake2b|cdc_scan" --pmc FETCH_SIZE SQ_INSTS_VALU -d gpurun_out/pmc_fetch -o p --output-format csv -- python bench.py --steps 2 --warmup 1 $B > gpurun_out/pmc_fetch.log 2>&1 && \
python tools/traffic.py gpurun_out/pmc_fetch gpurun_out/traffic.json > gpurun_out/traffic.log 2>&1 && \
timeout -k 10 400 python bench.py --traffic-json gpurun_out/traffic.json > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats -o run --output-format csv -- python bench.py --steps 20 --warmup 5 $B > gpurun_out/prof_stats.log 2>&1 && \
timeout -k 10 300 python bench.py --config c3 --steps 4 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/bench_c3.json 2>&1 && \
timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/bench_c4.json 2>&1 && \
PFS_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --group 8 --steps 3 --warmup 1 $B > gpurun_out/c2_n2_g8.json 2> gpurun_out/c2_n2_g8.err
rc=$?
echo rc=$rc
exit $rc
