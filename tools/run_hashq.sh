# gpu tests + bench sweep over launch-group size
mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 && \
for g in 1 4 16 32; do
  timeout -k 10 300 python bench.py --group $g --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/bench_g$g.json 2> gpurun_out/bench_g$g.err || exit 1
done && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_q -o run --output-format csv -- python bench.py --group 16 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/prof_q.log 2>&1
echo rc=$?
