#!/bin/bash
# configs1_literal's many-in-flight leg (one configs[1] batch per call, several calls in
# flight on their own contexts): batches in flight x the scan's workgroup cap, same box.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/${1:-r5lit}
mkdir -p $o
B="--no-cpu-baseline --no-e2e --no-pipelined --no-chain-floor --steps 2 --warmup 1 --group 8"
i=0
for v in "12 -1" "12 64" "20 -1" "20 64" "24 64" "12 -1" "20 64"; do
  i=$((i + 1)); set -- $v
  timeout -k 10 300 python bench.py $B --literal-inflight $1 --literal-scan-grid $2 > $o/lit_$1_$2_$i.json 2> $o/lit_$1_$2_$i.err || exit 1
done
python - $o <<'PY'
import json, sys, glob
o = sys.argv[1]
for f in sorted(glob.glob(o + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    m = d["configs1_literal"]["many_in_flight"]
    print(f.split("/")[-1], m["batches_in_flight"], m["scan_grid"], m["value"])
PY
