#!/bin/bash
# N=1 vs N=2/3 (every rank on the box's one GPU, gloo collectives) of the sharded forms:
# the index / chunk / fileset digests printed by bench.py must agree across N.
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/rehearse
mkdir -p $out
run1() { timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-literal "$@"; }
runN() { n=$1; shift; PFS_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench.py --gpus $n --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-literal "$@"; }
run1 --config c3 --inflight 1 > $out/c3_n1.json &&
runN 2 --config c3 > $out/c3_n2.json &&
runN 3 --config c3 > $out/c3_n3.json &&
run1 --config c4 --group 1 > $out/c4_n1.json &&
runN 2 --config c4 --group 1 > $out/c4_n2.json &&
run1 --path commit --config c4 > $out/commit_c4_n1.json &&
runN 2 --path commit --config c4 > $out/commit_c4_n2.json &&
run1 --path uw --config c4 --uw-bytes 6000000000 > $out/uw_c4_n1.json &&
runN 3 --path uw --config c4 --uw-bytes 6000000000 > $out/uw_c4_n3.json
rc=$?
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/rehearse/*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:
        print(f, "unreadable", e); continue
    dig = {k: d[k] for k in d if k.endswith("digest") or k in ("index_segments",)}
    print(f.split("/")[-1], d.get("n_gpus"), d.get("value"), d.get("ms_per_step"), dig)
PY
exit $rc
