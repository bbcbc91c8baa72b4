#!/bin/bash
# Four ranks on the one GPU through bench.py's own launcher (gloo, PFS_BENCH_REHEARSE=1), the
# default c2 line at 4 batches per rank against one GPU at 16 batches: equal index digests.
set -o pipefail
cd "$(dirname "$0")/.."
o=gpurun_out/rehearse4n4
mkdir -p $o
L="--steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-literal --no-pipelined --no-chain-floor"
timeout -k 10 300 python bench.py $L --group 16 > $o/c2_g16_n1.json 2> $o/c2_g16_n1.err &&
PFS_BENCH_REHEARSE=1 timeout -k 10 500 python bench.py --gpus 4 $L --group 4 > $o/c2_g4_n4.json 2> $o/c2_g4_n4.err &&
python - <<'PY'
import json
for f in ("c2_g16_n1", "c2_g4_n4"):
    d = json.loads(open("gpurun_out/rehearse4n4/%s.json" % f).read().strip().splitlines()[-1])
    print(f, d["n_gpus"], d["value"], d["ms_per_step"], d["index_digest"], d["index_segments"], d.get("index_gather"))
PY
