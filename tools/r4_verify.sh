#!/bin/bash
# Round 4: the driver's sequence (GPU suite, smoke(), default bench line) on the current tree,
# then the N>1 launch as the driver would call it (python bench.py --gpus 2, no launcher; two
# gloo ranks sharing the one GPU under PFS_BENCH_REHEARSE=1) beside N=1 at the same files
# (--group 16 = 2 x 8 batches): the c2 index digests must be equal.
set -o pipefail
cd "$(dirname "$0")/.."
o=gpurun_out/${1:-r4v}
mkdir -p $o
summ() { python - "$@" <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d.get("kernel_ms", {})
    print(f.split("/")[-1], d["n_gpus"], d["value"], d["ms_per_step"], round(k.get("scan", 0), 2),
          round(k.get("hash", 0), 2), round(k.get("scan_mhz", 0)), round(k.get("hash_mhz", 0)),
          d["roofline"]["frac"], d.get("index_digest"), d.get("index_segments"),
          d.get("index_gather"), d.get("parity"), d.get("cpu_baseline", {}).get("value"))
PY
}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $o/pytest_gpu.log 2>&1 && tail -1 $o/pytest_gpu.log &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 && tail -1 $o/smoke.log &&
timeout -k 10 400 python bench.py > $o/bench.json 2> $o/bench.err && summ $o/bench.json &&
timeout -k 10 300 python bench.py --group 16 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e \
    --no-literal --no-pipelined --no-chain-floor > $o/c2_g16_n1.json 2> $o/c2_g16_n1.err &&
PFS_BENCH_REHEARSE=1 timeout -k 10 400 python bench.py --gpus 2 --group 8 --steps 3 --warmup 1 \
    --no-cpu-baseline --no-e2e --no-literal --no-pipelined > $o/c2_g8_n2.json 2> $o/c2_g8_n2.err &&
summ $o/c2_g16_n1.json $o/c2_g8_n2.json
