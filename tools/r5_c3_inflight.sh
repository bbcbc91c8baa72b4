#!/bin/bash
# c3 (one 10 GiB stream per step): streams in flight 12 (default) vs 16, 20 and 24 on the
# 32 hardware queues, same box; the steps rule gives each run 2S timed steps.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/${1:-r5c3}
mkdir -p $o
i=0
for s in ${SWEEP:-12 16 20 24}; do
  i=$((i + 1))
  timeout -k 10 400 python bench.py --config c3 --inflight $s --steps 4 --warmup 2 --no-cpu-baseline --no-chain-floor > $o/c3_s${s}_$i.json 2> $o/c3_s${s}_$i.err || exit 1
done
python - $o <<'PY'
import json, sys, glob
o = sys.argv[1]
for f in sorted(glob.glob(o + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d.get("steps"), d.get("value"), (d.get("steady_state") or {}).get("value"), d.get("index_digest"))
PY
