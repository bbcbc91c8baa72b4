#!/bin/bash
# uw_stream_ab.sh's streaming forms with the scan's workgroups capped (PFSCDC_SCAN_GRID), so a
# group's scan never waits for CUs that other groups' chain-bound hashes hold.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/${1:-uwab2}
mkdir -p $o
B="--path uw --config c4 --uw-bytes 34359738368 --steps 2 --warmup 1 --no-cpu-baseline"
run() { name=$1; shift; timeout -k 10 240 python bench.py $B "$@" > $o/$name.json 2> $o/$name.err && \
  python -c "import json,sys; d=json.load(open('$o/$name.json')); print('$name', d['value'], d['ms_per_step'], d['commit_filesets_digest'], d['stages_ms'])"; }
run default &&
PFSCDC_SCAN_GRID=64 run g1e9_w4_sg64 --uw-group 1000000000 --uw-workers 4 &&
PFSCDC_SCAN_GRID=64 GPU_MAX_HW_QUEUES=32 run g1e9_w8_sg64_q32 --uw-group 1000000000 --uw-workers 8 &&
PFSCDC_SCAN_GRID=64 run g4e9_w4_sg64 --uw-group 4000000000 --uw-workers 4 &&
PFSCDC_SCAN_GRID=64 run g8e9_w2_sg64 --uw-group 8000000000 --uw-workers 2 &&
PFSCDC_SCAN_GRID=64 run g16e9_w2_sg64 --uw-group 16000000000 --uw-workers 2 &&
run default2
