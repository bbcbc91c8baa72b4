#!/bin/bash
# The host-fed writer (32 GiB c4 Put) with its serialized filesets written as they land: one
# fileset per group write (PFSCDC_UW_INFLIGHT = 1e9) or a few, on several group writers, against
# the default (one 32 GiB group after the Puts).  Same box, the default first and last.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/${1:-uwab}
mkdir -p $o
B="--path uw --config c4 --uw-bytes 34359738368 --steps 2 --warmup 1 --no-cpu-baseline"
run() { name=$1; shift; timeout -k 10 240 python bench.py $B "$@" > $o/$name.json 2> $o/$name.err && \
  python -c "import json,sys; d=json.load(open('$o/$name.json')); print('$name', d['value'], d['ms_per_step'], d['commit_filesets_digest'], d['stages_ms'])"; }
run default &&
run g1e9_w2 --uw-group 1000000000 --uw-workers 2 &&
run g1e9_w4 --uw-group 1000000000 --uw-workers 4 &&
run g2e9_w4 --uw-group 2000000000 --uw-workers 4 &&
run g4e9_w4 --uw-group 4000000000 --uw-workers 4 &&
GPU_MAX_HW_QUEUES=32 run g1e9_w8_q32 --uw-group 1000000000 --uw-workers 8 &&
GPU_MAX_HW_QUEUES=32 run g2e9_w4_q32 --uw-group 2000000000 --uw-workers 4 &&
run g8e9_w2 --uw-group 8000000000 --uw-workers 2 &&
run default2
