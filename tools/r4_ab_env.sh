#!/bin/bash
# Same-box A/B of an environment knob: alternate A and B runs of one bench command, print per
# run the value, step ms, the c2 kernels' times and clocks (or the uw/commit stages) and the
# digests.  Default bench arguments: the c2 line one step at a time without side legs.
# usage: tools/r4_ab_env.sh OUTDIR "ENV_A" "ENV_B" [reps] [bench args...]
set -o pipefail
cd "$(dirname "$0")/.."
o=gpurun_out/$1
A=$2
B=$3
reps=${4:-3}
shift 4 2>/dev/null || shift $#
args=("$@")
[ ${#args[@]} -eq 0 ] && args=(--steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-literal --no-pipelined --no-chain-floor)
mkdir -p $o
for i in $(seq 1 $reps); do
  for arm in A B; do
    if [ $arm = A ]; then e=$A; else e=$B; fi
    env $e timeout -k 10 300 python bench.py "${args[@]}" > $o/${arm}_$i.json 2> $o/${arm}_$i.err || exit 1
    python - $o/${arm}_$i.json "$arm[$e]" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d.get("kernel_ms", {})
out = [sys.argv[2], d["value"], d["ms_per_step"]]
if "scan_mhz" in k:
    out += ["scan", round(k["scan"], 3), round(k["scan_mhz"]), "hash", round(k["hash"], 3),
            round(k["hash_mhz"]), "frac", d["roofline"]["frac"]]
elif k:
    out += [{a: round(b, 1) for a, b in k.items()}]
if "stages_ms" in d:
    out += [d["stages_ms"]]
out += [{a: b for a, b in d.items() if a.endswith("digest")}]
print(*out)
PY
  done
done
