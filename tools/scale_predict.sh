#!/bin/bash
# Per-GPU rate of one rank's share of an 8-GPU c4/c5 commit (rank 0 of 8, alone on this GPU)
# at 1..8 commits per step: the N=8 prediction (no data-path collective; the index gather
# is ~1 MB).  Also the share at N=2 and N=4 with the auto group.
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/scale
mkdir -p $out
B="--no-cpu-baseline --no-e2e --no-literal --steps 4 --warmup 1"
for g in 1 2 4 6 8; do
  timeout -k 10 300 python bench.py --config c4 --shard 0/8 --group $g $B > $out/c4_s0of8_g$g.json || exit $?
done
for n in 2 4 8; do
  timeout -k 10 300 python bench.py --config c4 --shard 0/$n $B > $out/c4_s0of${n}_auto.json || exit $?
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/scale/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    c = d["config"]
    print(f.split("/")[-1], c.get("commits_per_step"), d["value"], d["ms_per_step"],
          d["segments_per_step"], d["kernel_ms_median"].get("hash_span"))
PY
