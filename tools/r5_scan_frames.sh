#!/bin/bash
# (Historical: the exp/ builds it compares were deleted after the rejection; the two-frame
# patch is in profiles/r5/rejected/scan_two_frames/.)
# The two-frame narrow scan (round 5): same-box A/B on the default line, alternating.
# O / O8 = the one-frame form at 3 / 2 waves per SIMD; N8 = two frames, masked keys, 2 waves
# per SIMD (at 3 the ring needs two register sets and spills); X3 / X2 = two frames with the
# odd positions' keys masked by a separate AND, 3 / 2 waves per SIMD.  PARITY=1: GPU parity
# of this tree first.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/${1:-r5frames}
mkdir -p $o
B="--no-cpu-baseline --no-e2e --no-literal --no-pipelined --no-chain-floor"
if [ "${PARITY:-0}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_configs.py -x -q -m gpu --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
  tail -1 $o/pytest.log
fi
for i in 1 2 3; do
  for v in ${VARIANTS:-O O8 N8 X3 X2}; do
    case $v in N) L="";; *) L=exp/lib_$(echo $v | tr A-Z a-z).so;; esac
    [ $v = O ] && L=exp/lib_old.so
    PFSCDC_LIB=$L timeout -k 10 200 python bench.py --steps 6 --warmup 2 $B > $o/${v}_$i.json 2> $o/${v}_$i.err || exit 1
  done
done
python - $o <<'PY'
import json, sys, glob
o = sys.argv[1]
for f in sorted(glob.glob(o + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d.get("kernel_ms", {})
    print(f.split("/")[-1], d.get("value"), d.get("ms_per_step"), d.get("index_digest"),
          {a: round(b, 2) for a, b in k.items() if a in ("scan", "scan_span", "hash", "scan_mhz", "hash_mhz")})
PY
