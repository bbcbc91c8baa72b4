# gpu tests + bench (inflight 1) + kernel-trace stats of the bench
mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 > gpurun_out/bench_s1.json 2> gpurun_out/bench_s1.err && \
timeout -k 10 300 python bench.py --inflight 4 --steps 16 --no-cpu-baseline --no-e2e > gpurun_out/bench_s4.json 2> gpurun_out/bench_s4.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_k -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/prof_k.log 2>&1
echo rc=$?
