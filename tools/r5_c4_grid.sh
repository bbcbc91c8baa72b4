#!/bin/bash
# c4 / c5 (two commits in flight): scans full-width (default) vs capped at 64 workgroups,
# alternating, same box.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/${1:-r5c4grid}
mkdir -p $o
i=0
for v in "c4 0" "c4 64" "c5 0" "c5 64" "c4 0" "c4 64" "c5 0" "c5 64"; do
  i=$((i + 1)); set -- $v
  PFSCDC_SCAN_GRID=$2 timeout -k 10 400 python bench.py --config $1 --steps 4 --warmup 2 --no-cpu-baseline --no-chain-floor > $o/$1_g$2_$i.json 2> $o/$1_g$2_$i.err || exit 1
done
python - $o <<'PY'
import json, sys, glob
o = sys.argv[1]
for f in sorted(glob.glob(o + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d.get("steps"), d.get("value"), (d.get("steady_state") or {}).get("value"), d.get("index_digest"))
PY
