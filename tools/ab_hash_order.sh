#!/bin/bash
# A/B: steps in flight with the hash kernels serialized vs free to share the CUs, plus a
# kernel-trace pass of the serialized form (its per-launch durations vs the in-kernel spans).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab_order && export TMPDIR=/tmp
B="--no-cpu-baseline --no-e2e --no-literal --steps 20 --warmup 5"
for i in 1 2; do
  timeout -k 10 200 python bench.py $B --hash-order serial > gpurun_out/ab_order/serial_$i.json || exit $?
  timeout -k 10 200 python bench.py $B --hash-order free > gpurun_out/ab_order/free_$i.json || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_order/prof_serial -o run --output-format csv -- python bench.py $B --hash-order serial > gpurun_out/ab_order/prof_serial.log 2>&1 || exit $?
python - <<'PY'
import json, glob, csv
for f in sorted(glob.glob("gpurun_out/ab_order/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d["kernel_ms"]["hash_span"], d["kernel_ms"]["scan_span"], d["kernel_ms"]["hash"])
for f in glob.glob("gpurun_out/ab_order/prof_serial/*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        print(r["Name"][:40], r["Calls"], r["AverageNs"], r["MinNs"], r["MaxNs"])
PY
