# bench: steps in flight x group size (quad kernel)
mkdir -p gpurun_out && export TMPDIR=/tmp && \
for cfg in ${CFGS:-"16 2" "24 2" "8 4"}; do
  set -- $cfg
  timeout -k 10 300 python bench.py --group $1 --inflight $2 --steps 8 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/bi_g$1_s$2.json 2> gpurun_out/bi_g$1_s$2.err || exit 1
done
echo rc=$?
