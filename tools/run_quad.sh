# gpu tests + bench sweep: args are group:waves_per_simd tokens (default 1:2 16:2 32:2)
mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || exit 1
for cfg in ${@:-1:2 16:2 32:2}; do
  g=${cfg%%:*}; w=${cfg##*:}
  PFSCDC_HASH_WAVES=$w timeout -k 10 300 python bench.py --group $g --steps 4 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/bq_g${g}_w$w.json 2> gpurun_out/bq_g${g}_w$w.err || exit 1
done
echo rc=$?
