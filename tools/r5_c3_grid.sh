#!/bin/bash
# c3 at twenty streams in flight: the scans' workgroup cap (PFSCDC_SCAN_GRID) 32 / 64 / 128,
# alternating, same box.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/${1:-r5c3grid}
mkdir -p $o
i=0
for g in 32 64 128 32 64 128; do
  i=$((i + 1))
  PFSCDC_SCAN_GRID=$g timeout -k 10 400 python bench.py --config c3 --steps 4 --warmup 2 --no-cpu-baseline --no-chain-floor > $o/c3_g${g}_$i.json 2> $o/c3_g${g}_$i.err || exit 1
done
python - $o <<'PY'
import json, sys, glob
o = sys.argv[1]
for f in sorted(glob.glob(o + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d.get("steps"), d.get("value"), (d.get("steady_state") or {}).get("value"), d["config"].get("scan_grid"))
PY
