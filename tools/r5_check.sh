#!/bin/bash
# Round 5 check of the tree as it stands: the GPU suite, smoke(), a short default line and the
# commit digests (c4 commit G=2, uw 8 GiB) that must not move when the library changes form.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/${1:-r5chk}
mkdir -p $o
B="--no-cpu-baseline --no-e2e --no-literal --no-pipelined --no-chain-floor"
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $o/pytest_gpu.log 2>&1 && tail -1 $o/pytest_gpu.log &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 && tail -1 $o/smoke.log &&
timeout -k 10 300 python bench.py --steps 6 --warmup 2 $B > $o/bench_short.json 2> $o/bench_short.err &&
timeout -k 10 300 python bench.py --path commit --config c4 --group 2 --steps 3 --warmup 1 --no-cpu-baseline > $o/commit_c4_g2.json 2> $o/commit_c4_g2.err &&
timeout -k 10 300 python bench.py --path uw --config c4 --steps 2 --warmup 1 > $o/uw_c4_8g.json 2> $o/uw_c4_8g.err &&
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
    print(f.split("/")[-1], d.get("value"), d.get("ms_per_step"), d.get("roofline", {}).get("frac"),
          {a: round(b, 2) for a, b in k.items() if a in ("scan", "hash", "scan_mhz", "hash_mhz", "create")},
          {a: b for a, b in d.items() if a.endswith("digest")}, d.get("config", {}).get("scan_skip"))
PY
