#!/bin/bash
# Same-box A/B: the round-4 tree (ab_r4/, built from commit 73aee90) against this tree on the
# default line, alternating; then this tree's c3 line under the steps-in-flight rule and the
# eight-rank gloo rehearsal of the N > 1 lines (every rank on the one GPU).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/${1:-r5ab}
mkdir -p $o
B="--no-cpu-baseline --no-e2e --no-literal --no-pipelined --no-chain-floor"
for i in 1 2 3; do
  (cd ab_r4 && timeout -k 10 200 python bench.py --steps 6 --warmup 2 $B) > $o/A_$i.json 2> $o/A_$i.err || exit 1
  timeout -k 10 200 python bench.py --steps 6 --warmup 2 $B > $o/B_$i.json 2> $o/B_$i.err || exit 1
done
timeout -k 10 300 python bench.py --config c3 --steps 4 --warmup 2 --no-cpu-baseline > $o/c3.json 2> $o/c3.err || exit 1
timeout -k 10 300 python bench.py $B --steps 2 --warmup 1 --group 16 > $o/c2_g16_n1.json 2> $o/c2_g16_n1.err || exit 1
PFS_BENCH_REHEARSE=1 timeout -k 10 600 python bench.py --gpus 8 $B --steps 2 --warmup 1 --group 2 > $o/c2_g2_n8.json 2> $o/c2_g2_n8.err || exit 1
PFS_BENCH_REHEARSE=1 timeout -k 10 600 python bench.py --gpus 8 --config c4 --group 1 --inflight 1 $B --steps 2 --warmup 1 > $o/c4_g1_n8.json 2> $o/c4_g1_n8.err || exit 1
python - $o <<'PY'
import json, sys, glob
o = sys.argv[1]
for f in sorted(glob.glob(o + "/*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:
        print(f, "unreadable", e)
        continue
    k = d.get("kernel_ms", {})
    print(f.split("/")[-1], d.get("n_gpus"), d.get("steps"), d.get("value"), d.get("ms_per_step"),
          {a: round(b, 2) for a, b in k.items() if a in ("scan", "hash", "scan_mhz", "hash_mhz")},
          d.get("index_digest"), (d.get("parity") or {}).get("gpu_equals_cpu_oracle"),
          (d.get("index_gather") or {}).get("moved_over_live"), d.get("steady_state"))
PY
