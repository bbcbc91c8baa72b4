#!/bin/bash
# Same-box sweep of the hash's fair-share knobs on the default line, alternating with the
# defaults (PFSCDC_HASH_FAIR=1, PFSCDC_HASH_FAIR_EVERY=256).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/${1:-r5knobs}
mkdir -p $o
B="--no-cpu-baseline --no-e2e --no-literal --no-pipelined --no-chain-floor"
for i in 1 2; do
  for v in def e64 e1024 nofair; do
    case $v in def) E="";; e64) E="PFSCDC_HASH_FAIR_EVERY=64";; e1024) E="PFSCDC_HASH_FAIR_EVERY=1024";; nofair) E="PFSCDC_HASH_FAIR=0";; esac
    env $E timeout -k 10 200 python bench.py --steps 8 --warmup 2 $B > $o/${v}_$i.json 2> $o/${v}_$i.err || exit 1
  done
done
python - $o <<'PY'
import json, sys, glob
o = sys.argv[1]
for f in sorted(glob.glob(o + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d.get("kernel_ms", {})
    print(f.split("/")[-1], d.get("value"), d.get("ms_per_step"), {a: round(b, 2) for a, b in k.items() if a in ("scan", "hash", "hash_span", "hash_mhz")})
PY
