#!/bin/bash
# Same-box A/B/C/... of environment settings: each round runs every arm once, in order.
# usage: tools/r4_ab_multi.sh OUTDIR reps "ENV_1" "ENV_2" ... [-- bench args...]
set -o pipefail
cd "$(dirname "$0")/.."
o=gpurun_out/$1
reps=$2
shift 2
arms=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do arms+=("$1"); shift; done
[ "$1" = "--" ] && shift
args=("$@")
[ ${#args[@]} -eq 0 ] && args=(--steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-literal --no-pipelined --no-chain-floor)
mkdir -p $o
for i in $(seq 1 $reps); do
  for k in "${!arms[@]}"; do
    e=${arms[$k]}
    env $e timeout -k 10 300 python bench.py "${args[@]}" > $o/arm${k}_$i.json 2> $o/arm${k}_$i.err || exit 1
    python - $o/arm${k}_$i.json "$k[$e]" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d.get("kernel_ms", {})
out = [sys.argv[2], d["value"], d["ms_per_step"]]
if "scan_mhz" in k:
    out += ["scan", round(k["scan"], 3), "span", round(k.get("scan_span", 0), 3), round(k["scan_mhz"]),
            "hash", round(k["hash"], 3), round(k["hash_mhz"]), "frac", d["roofline"]["frac"],
            "rolled", d.get("roofline_cdc", {}).get("rolled_fraction")]
elif k:
    out += [{a: round(b, 1) for a, b in k.items()}]
if "stages_ms" in d:
    out += [d["stages_ms"]]
out += [{a: b for a, b in d.items() if a.endswith("digest")}]
print(*out)
PY
  done
done
