#!/bin/bash
# Round 6: the host-fed writer (32 GiB c4 Put) on one ctx and over device groups of 1, 2 and 4
# ctxs on the one GPU; the filesets digest must not change.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/${1:-r6uwg}
mkdir -p $o
B="--path uw --config c4 --uw-bytes 34359738368 --steps 2 --warmup 1 --no-cpu-baseline"
run() { name=$1; shift; timeout -k 10 300 python bench.py $B "$@" > $o/$name.json 2> $o/$name.err && \
  python -c "import json; d=json.load(open('$o/$name.json')); print('$name', d['value'], d['ms_per_step'], d['commit_filesets_digest'], d['config']['parallelism'])"; }
run one && run m1 --members 0 && run m2 --members 0,0 && run m4 --members 0,0,0,0 && run one2
