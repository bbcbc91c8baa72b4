#!/bin/bash
# Round 3 rehearsal of the N>1 paths on the one GPU (gloo collectives, two ranks sharing the
# card) with the final tree: the default c2 line at N=2 (8 batches per rank), c4 put and the
# commit data plane at N=1 vs N=2 (digests must agree across N).
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/rehearse3b
mkdir -p $out
run1() { timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-literal "$@"; }
runN() { n=$1; shift; PFS_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench.py --gpus $n --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-literal "$@"; }
runN 2 --group 8 --no-pipelined > $out/c2_n2_g8.json &&
run1 --config c4 --inflight 1 > $out/c4_n1.json &&
runN 2 --config c4 --group 2 --inflight 1 > $out/c4_n2.json &&
run1 --path commit --config c4 --group 1 > $out/commit_c4_n1.json &&
runN 2 --path commit --config c4 --group 1 > $out/commit_c4_n2.json
rc=$?
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/rehearse3b/*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:
        print(f, "unreadable", e); continue
    dig = {k: d[k] for k in d if k.endswith("digest") or k in ("index_segments",)}
    print(f.split("/")[-1], d.get("n_gpus"), d.get("value"), d.get("ms_per_step"), d.get("scaling"),
          d.get("single_commit", {}).get("value"), dig)
PY
exit $rc
