#!/bin/bash
# Round-4 rehearsal of the N>1 paths on the one GPU, launched the way the driver's plain
# `python bench.py --gpus N` is (bench.py starts torch.distributed.run itself), two gloo ranks
# sharing the card (PFS_BENCH_REHEARSE=1): digests must equal N=1's.
set -o pipefail
cd "$(dirname "$0")/.."
o=gpurun_out/rehearse4
mkdir -p $o
L="--steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-literal --no-pipelined --no-chain-floor"
run1() { out=$1; shift; timeout -k 10 300 python bench.py $L "$@" > $o/$out.json 2> $o/$out.err; }
runN() { out=$1; n=$2; shift 2; PFS_BENCH_REHEARSE=1 timeout -k 10 420 python bench.py --gpus $n $L "$@" > $o/$out.json 2> $o/$out.err; }
run1 c4_n1 --config c4 --inflight 1 &&
runN c4_n2 2 --config c4 --group 1 --inflight 1 &&
run1 commit_c4_n1 --path commit --config c4 --group 1 &&
runN commit_c4_n2 2 --path commit --config c4 --group 1 &&
run1 c2_g16_n1 --group 16 &&
runN c2_g8_n2 2 --group 8
rc=$?
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/rehearse4/*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:
        print(f, "unreadable", e); continue
    dig = {k: d[k] for k in d if k.endswith("digest") or k in ("index_segments",)}
    print(f.split("/")[-1], d.get("n_gpus"), d.get("value"), d.get("ms_per_step"), d.get("scaling"),
          d.get("index_gather", {}).get("moved_over_live"), dig)
PY
exit $rc
