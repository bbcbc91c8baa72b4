# gpu tests + bench sweep (lane kernel): group size x waves per SIMD
mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 && \
for cfg in "1 2" "8 2" "16 1" "16 2" "16 3" "32 2"; do
  set -- $cfg
  PFSCDC_HASH_WAVES=$2 timeout -k 10 300 python bench.py --group $1 --steps 4 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/bl_g$1_w$2.json 2> gpurun_out/bl_g$1_w$2.err || exit 1
done
echo rc=$?
