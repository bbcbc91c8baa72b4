#!/bin/bash
# Round-3 artifacts: GPU tests, smoke, PMC pass (FETCH_SIZE + SQ_INSTS_VALU per launch ->
# traffic json), the default bench line, a kernel-trace --stats pass of the bench's 128 GiB
# steps, c3 / c4 lines, and the per-GPU scale prediction (rank 0's share of N = 8 at G = 1..8).
set -o pipefail
cd "$(dirname "$0")/.."
o=gpurun_out/r3f
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
bash tools/scale_predict.sh > $o/scale_predict.txt 2>&1
rc=$?
python - <<'PY'
import json
for f in ("bench", "bench_c4", "bench_c3"):
    try:
        d = json.loads(open("gpurun_out/r3f/%s.json" % f).read().strip().splitlines()[-1])
    except Exception as e:
        print(f, "unreadable", e); continue
    k = d["kernel_ms"]
    print(f, d["value"], d["ms_per_step"], round(k["scan"], 2), round(k["hash"], 2), round(k.get("scan_mhz", 0)),
          round(k.get("hash_mhz", 0)), d["roofline"]["frac"], d["roofline"]["traffic"], d.get("parity"),
          d.get("cpu_baseline", {}).get("value"))
PY
grep json gpurun_out/r3f/scale_predict.txt
echo rc=$rc
exit $rc
