#!/bin/bash
# Round-3 artifacts of the final tree (hash bins + fair share, two-set commit, c3 four streams
# in flight): GPU tests, smoke, PMC pass (FETCH_SIZE + SQ_INSTS_VALU per launch -> traffic
# json), the default bench line with that traffic, a kernel-trace --stats pass of the bench's
# 128 GiB steps, c3 / c4 lines, the c4 commit data plane at G=2.
set -o pipefail
cd "$(dirname "$0")/.."
o=gpurun_out/r3f4
mkdir -p $o && export TMPDIR=/tmp
B="--no-cpu-baseline --no-e2e --no-literal --no-pipelined --no-chain-floor"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $o/pytest_gpu.log 2>&1 && tail -1 $o/pytest_gpu.log && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 && tail -1 $o/smoke.log && \
timeout -k 10 240 rocprofv3 --kernel-include-regex "blake2b|cdc_scan" --pmc FETCH_SIZE SQ_INSTS_VALU -d $o/pmc_fetch -o p --output-format csv -- python bench.py --steps 2 --warmup 1 $B > $o/pmc_fetch.log 2>&1 && \
python tools/traffic.py $o/pmc_fetch $o/traffic_c2.json > $o/traffic.log 2>&1 && cat $o/traffic.log && \
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --traffic-json $o/traffic_c2.json > $o/bench.json 2> $o/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof_stats -o run --output-format csv -- python bench.py --steps 20 --warmup 5 $B > $o/prof_stats.log 2>&1 && \
timeout -k 10 300 python bench.py --config c4 --steps 4 --warmup 1 > $o/bench_c4.json 2> $o/bench_c4.err && \
timeout -k 10 300 python bench.py --config c3 --steps 4 --warmup 1 > $o/bench_c3.json 2> $o/bench_c3.err && \
timeout -k 10 400 python bench.py --config c4 --path commit --group 2 --steps 3 --warmup 1 > $o/commit_c4_g2.json 2> $o/commit_c4_g2.err
rc=$?
python - <<'PY'
import json
for f in ("bench", "bench_c4", "bench_c3", "commit_c4_g2"):
    try:
        d = json.loads(open("gpurun_out/r3f4/%s.json" % f).read().strip().splitlines()[-1])
    except Exception as e:
        print(f, "unreadable", e); continue
    k = d["kernel_ms"]
    print(f, d["value"], d["ms_per_step"], {a: round(b, 2) for a, b in k.items() if isinstance(b, float)},
          d["roofline"]["frac"], d["roofline"].get("traffic"), d.get("parity"),
          d.get("cpu_baseline", {}).get("value"), d.get("one_step_alone"))
PY
echo rc=$rc
exit $rc
