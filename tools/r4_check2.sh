#!/bin/bash
# A short default line (the config now carries the scan's skip settings) and two gloo ranks
# on the one GPU through bench.py's own launcher; digests equal to one GPU's.
set -o pipefail
cd "$(dirname "$0")/.."
o=gpurun_out/r4chk2
mkdir -p $o
L="--steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-literal --no-pipelined --no-chain-floor"
timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline > $o/bench_short.json 2> $o/bench_short.err &&
timeout -k 10 300 python bench.py $L --group 16 > $o/c2_g16_n1.json 2> $o/c2_g16_n1.err &&
PFS_BENCH_REHEARSE=1 timeout -k 10 400 python bench.py --gpus 2 $L --group 8 > $o/c2_g8_n2.json 2> $o/c2_g8_n2.err &&
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r4chk2/bench_short.json").read().strip().splitlines()[-1])
print("short", d["value"], d["config"]["scan_skip"])
for f in ("c2_g16_n1", "c2_g8_n2"):
    d = json.loads(open("gpurun_out/r4chk2/%s.json" % f).read().strip().splitlines()[-1])
    print(f, d["n_gpus"], d["value"], d["index_digest"], (d.get("index_gather") or {}).get("moved_over_live"))
PY
