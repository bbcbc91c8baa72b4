# gpu tests + bench at inflight 1 and 8 + kernel-trace profile
mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/t_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --inflight 1 > gpurun_out/bench_s1.json 2> gpurun_out/bench_s1.err && \
timeout -k 10 300 python bench.py --inflight 8 --no-cpu-baseline --no-e2e > gpurun_out/bench_s8.json 2> gpurun_out/bench_s8.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_k -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/prof_k.log 2>&1
echo rc=$?
