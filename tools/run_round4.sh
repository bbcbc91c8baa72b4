#!/bin/bash
# Round-4 artifacts of the final tree: the GPU suite, smoke(), the PMC pass of the default
# line (FETCH_SIZE + SQ_INSTS_VALU per launch -> traffic_c2.json), the default bench line, a
# kernel-trace --stats pass of the same 128 GiB steps (no side legs, so every blake2b/scan
# launch is one step's), then the other configurations' lines.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/${1:-r4final}
mkdir -p $o
B="--no-cpu-baseline --no-e2e --no-literal --no-pipelined --no-chain-floor"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $o/pytest_gpu.log 2>&1 && tail -1 $o/pytest_gpu.log &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 && tail -1 $o/smoke.log &&
timeout -s KILL 240 rocprofv3 --kernel-include-regex "blake2b|cdc_scan" --pmc FETCH_SIZE SQ_INSTS_VALU -d $o/pmc -o p --output-format csv -- python3 bench.py --steps 2 --warmup 1 $B > $o/pmc.log 2>&1 &&
python tools/traffic.py $o/pmc $o/traffic_c2.json > $o/traffic.log 2>&1 && cat $o/traffic.log &&
timeout -k 10 400 python bench.py --traffic-json $o/traffic_c2.json > $o/bench.json 2> $o/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/stats -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 $B > $o/stats_bench.json 2> $o/stats.err &&
timeout -k 10 300 python bench.py --config c3 --steps 4 --warmup 2 --no-cpu-baseline > $o/bench_c3.json 2> $o/bench_c3.err &&
timeout -k 10 300 python bench.py --config c4 --steps 4 --warmup 2 --no-cpu-baseline > $o/bench_c4.json 2> $o/bench_c4.err &&
timeout -k 10 300 python bench.py --path commit --config c4 --group 2 --steps 3 --warmup 1 --no-cpu-baseline > $o/commit_c4_g2.json 2> $o/commit_c4_g2.err &&
timeout -k 10 300 python bench.py --path uw --config c4 --uw-bytes 34359738368 --steps 2 --warmup 1 > $o/uw_c4_32g.json 2> $o/uw_c4_32g.err &&
python - $o <<'PY'
import json, sys, glob
o = sys.argv[1]
for f in sorted(glob.glob(o + "/*.json")):
    if f.endswith("traffic_c2.json"):
        continue
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:
        print(f, "unreadable", e)
        continue
    k = d.get("kernel_ms", {})
    print(f.split("/")[-1], d.get("value"), d.get("ms_per_step"), d.get("roofline", {}).get("frac"),
          {a: round(b, 2) for a, b in k.items() if a in ("scan", "hash", "scan_mhz", "hash_mhz", "create")},
          {a: b for a, b in d.items() if a.endswith("digest")})
PY
