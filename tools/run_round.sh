# Round artifacts: gpu tests, PMC FETCH_SIZE pass (traffic), default bench, kernel-trace stats.
mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-include-regex "blake2b|cdc_scan" --pmc FETCH_SIZE SQ_INSTS_VALU -d gpurun_out/pmc_fetch -o p --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/pmc_fetch.log 2>&1 && \
python tools/traffic.py gpurun_out/pmc_fetch gpurun_out/traffic.json > gpurun_out/traffic.log 2>&1 && \
timeout -k 10 400 python bench.py --traffic-json gpurun_out/traffic.json > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/prof_stats.log 2>&1
echo rc=$?
