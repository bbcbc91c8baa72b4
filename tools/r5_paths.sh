#!/bin/bash
# The bench paths the final run does not cover, through the split bench (benchkit/): chunk.Get,
# the re-chunk path, one shard alone, the c3 stream split over two gloo ranks on the one GPU
# (digest and border parity against one GPU), and c5 over two ranks (sample parity).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/${1:-r5paths}
mkdir -p $o
B="--no-cpu-baseline --no-e2e --no-literal --no-pipelined --no-chain-floor"
timeout -k 10 300 python bench.py --path get --steps 3 --warmup 1 $B > $o/get.json 2> $o/get.err &&
timeout -k 10 300 python bench.py --path rechunk --steps 2 --warmup 1 > $o/rechunk.json 2> $o/rechunk.err &&
timeout -k 10 300 python bench.py --config c4 --shard 0/8 --steps 3 --warmup 1 $B > $o/c4_shard0of8.json 2> $o/c4_shard0of8.err &&
PFS_BENCH_REHEARSE=1 timeout -k 10 400 python bench.py --gpus 2 --config c3 --steps 2 --warmup 1 $B > $o/c3_n2.json 2> $o/c3_n2.err &&
PFS_BENCH_REHEARSE=1 timeout -k 10 400 python bench.py --gpus 2 --config c5 --group 1 --inflight 1 --steps 2 --warmup 1 $B > $o/c5_n2.json 2> $o/c5_n2.err &&
timeout -k 10 300 python bench.py --config c5 --group 1 --inflight 1 --steps 2 --warmup 1 $B > $o/c5_n1.json 2> $o/c5_n1.err &&
python - $o <<'PY'
import json, sys, glob
o = sys.argv[1]
for f in sorted(glob.glob(o + "/*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:
        print(f, "unreadable", e)
        continue
    print(f.split("/")[-1], d.get("n_gpus"), d.get("value"), d.get("ms_per_step"),
          {a: b for a, b in d.items() if a.endswith("digest")}, d.get("parity"), d.get("dedup"))
PY
