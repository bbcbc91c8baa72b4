#!/bin/bash
# Artifacts of the final tree: what the driver runs (GPU suite, smoke(), the default
# line), the PMC pass of the default line (FETCH_SIZE + SQ_INSTS_VALU per launch ->
# traffic_c2.json), the default line reading it, a kernel-trace --stats pass of the same 128 GiB
# steps (no side legs, so every blake2b/scan launch is one step's), then the other
# configurations' lines, the device group and the eight-rank rehearsal.
#   bash tools/final.sh NAME   (on the GPU box; output under gpurun_out/NAME)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/${1:-final}
mkdir -p $o
B="--no-cpu-baseline --no-e2e --no-literal --no-pipelined --no-chain-floor"
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $o/pytest_gpu.log 2>&1 && tail -1 $o/pytest_gpu.log &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 && tail -1 $o/smoke.log &&
timeout -k 10 400 python bench.py > $o/bench_driverlike.json 2> $o/bench_driverlike.err &&
timeout -s KILL 240 rocprofv3 --kernel-include-regex "blake2b|cdc_scan" --pmc FETCH_SIZE SQ_INSTS_VALU -d $o/pmc -o p --output-format csv -- python3 bench.py --steps 2 --warmup 1 $B > $o/pmc.log 2>&1 &&
python tools/traffic.py $o/pmc $o/traffic_c2.json > $o/traffic.log 2>&1 && cat $o/traffic.log &&
timeout -k 10 400 python bench.py --traffic-json $o/traffic_c2.json > $o/bench.json 2> $o/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/stats -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 $B > $o/stats_bench.json 2> $o/stats.err &&
timeout -k 10 300 python bench.py --config c3 --steps 4 --warmup 2 --no-cpu-baseline > $o/bench_c3.json 2> $o/bench_c3.err &&
timeout -k 10 300 python bench.py --config c4 --steps 4 --warmup 2 --no-cpu-baseline > $o/bench_c4.json 2> $o/bench_c4.err &&
timeout -k 10 300 python bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline > $o/bench_c5.json 2> $o/bench_c5.err &&
timeout -k 10 300 python bench.py --path commit --config c4 --group 2 --steps 3 --warmup 1 > $o/commit_c4_g2.json 2> $o/commit_c4_g2.err &&
timeout -k 10 300 python bench.py --path uw --config c4 --uw-bytes 34359738368 --steps 2 --warmup 1 > $o/uw_c4_32g.json 2> $o/uw_c4_32g.err &&
timeout -k 10 300 python bench.py --path group --members 0,0,0,0,0,0,0,0 --steps 5 --warmup 2 > $o/group_m8.json 2> $o/group_m8.err &&
PFS_BENCH_REHEARSE=1 timeout -k 10 600 python bench.py --gpus 8 $B --steps 2 --warmup 1 --group 2 > $o/c2_g2_n8.json 2> $o/c2_g2_n8.err &&
timeout -k 10 300 python bench.py $B --steps 2 --warmup 1 --group 16 > $o/c2_g16_n1.json 2> $o/c2_g16_n1.err &&
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
    print(f.split("/")[-1], d.get("n_gpus"), d.get("value"), d.get("ms_per_step"), d.get("roofline", {}).get("frac"),
          {a: round(b, 2) for a, b in k.items() if a in ("scan", "hash", "scan_mhz", "hash_mhz", "create")},
          {a: b for a, b in d.items() if a.endswith("digest")}, (d.get("parity") or {}).get("gpu_equals_cpu_oracle"),
          (d.get("steady_state") or {}).get("value"))
PY
