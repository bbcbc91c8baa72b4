# A/B: default lib vs an alternative lib (PFSCDC_LIB) on parity tests + bench at given groups
# usage: bash tools/run_ab.sh <alt.so> <group>...
mkdir -p gpurun_out && export TMPDIR=/tmp
ALT=$1; shift
PFSCDC_LIB=$ALT timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_alt.log 2>&1 || exit 1
for g in "$@"; do
  PFSCDC_LIB=$ALT timeout -k 10 300 python bench.py --group $g --steps 4 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/ab_alt_g$g.json 2> gpurun_out/ab_alt_g$g.err || exit 1
done
echo rc=$?
