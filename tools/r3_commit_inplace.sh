#!/bin/bash
# round 3: in-place ciphertext commit: GPU tests, then c4 commit at G=1 (copy / in place) and G=2
mkdir -p gpurun_out/r3
timeout -k 10 300 python -u -m pytest tests/test_gpu_commit.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3/t_commit.log 2>&1 || { tail -30 gpurun_out/r3/t_commit.log; exit 1; }
tail -1 gpurun_out/r3/t_commit.log
for cfg in "1 0" "1 1" "2 -1"; do
  set -- $cfg
  timeout -k 10 400 python bench.py --config c4 --path commit --group $1 --in-place $2 --steps 3 --warmup 1 > gpurun_out/r3/c4_commit_g$1_ip$2.json 2> gpurun_out/r3/c4_commit_g$1_ip$2.err || { tail -5 gpurun_out/r3/c4_commit_g$1_ip$2.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r3/c4_commit_g$1_ip$2.json').read().strip().splitlines()[-1]); print('commit G=$1 ip=$2', d['config']['ciphertext_in_place'], d['value'], d['ms_per_step'], d['kernel_ms'], d.get('parity'), d['commit_chunks_digest'], d['dataref_hashes_digest'])"
done
