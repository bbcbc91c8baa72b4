#!/bin/bash
# (Historical: the PFS_EXP_ROT_ODD / PFS_EXP_COPIES16 builds it ran were deleted with the form;
# the two-frame patch is in profiles/r5/rejected/scan_two_frames/.)
# Timing-only probe of a pair-rotation scan form (wrong digests in B/C/D; only the scan's
# duration and clock matter): A = product; B = 16 table copies in use (2-way LDS bank
# conflicts); C = B + the state rotated at odd positions only (the VALU count of a form that
# rotates by 2 once per pair with per-parity pre-rotated tables); D = C's VALU with 32 copies.
# Alternating, same box.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/${1:-r5scanprobe}
mkdir -p $o
B="--no-cpu-baseline --no-e2e --no-literal --no-pipelined --no-chain-floor"
for i in 1 2 3; do
  for v in A B C D; do
    if [ $v = A ]; then L=""; else L=exp/lib_$v.so; fi
    PFSCDC_LIB=$L timeout -k 10 200 python bench.py --steps 6 --warmup 2 $B > $o/${v}_$i.json 2> $o/${v}_$i.err || exit 1
  done
done
python - $o <<'PY'
import json, sys, glob
o = sys.argv[1]
for f in sorted(glob.glob(o + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d.get("kernel_ms", {})
    print(f.split("/")[-1], d.get("value"), d.get("ms_per_step"),
          {a: round(b, 2) for a, b in k.items() if a in ("scan", "scan_span", "hash", "scan_mhz", "hash_mhz")})
PY
