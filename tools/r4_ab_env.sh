#!/bin/bash
# Same-box A/B of an environment knob on the default c2 line (one step at a time, no side
# legs): alternate A and B runs, print per run value / step ms / scan and hash ms and clocks.
# usage: tools/r4_ab_env.sh OUTDIR "ENV_A" "ENV_B" [reps] [extra bench args...]
set -o pipefail
cd "$(dirname "$0")/.."
o=gpurun_out/$1
A=$2
B=$3
reps=${4:-3}
shift 4 2>/dev/null || shift $#
mkdir -p $o
for i in $(seq 1 $reps); do
  for arm in A B; do
    if [ $arm = A ]; then e=$A; else e=$B; fi
    env $e timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e \
        --no-literal --no-pipelined --no-chain-floor "$@" > $o/${arm}_$i.json 2> $o/${arm}_$i.err || exit 1
    python - $o/${arm}_$i.json "$arm[$e]" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernel_ms"]
print(sys.argv[2], d["value"], d["ms_per_step"], "scan", round(k["scan"], 3), round(k["scan_mhz"]),
      "hash", round(k["hash"], 3), round(k["hash_mhz"]), "frac", d["roofline"]["frac"],
      d.get("index_digest"))
PY
  done
done
