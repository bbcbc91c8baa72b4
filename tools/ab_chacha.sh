#!/bin/bash
# round 3: ChaCha20 plaintext loads hidden under the rounds (A = previous build, B = this one)
# usage: bash tools/ab_chacha.sh <a.so> <b.so>
mkdir -p gpurun_out/r3/chacha
A=$1; B=$2
PFSCDC_LIB=$B timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_commit.py tests/test_gpu_refid.py tests/test_gpu_parity.py > gpurun_out/r3/chacha/t.log 2>&1 || { tail -20 gpurun_out/r3/chacha/t.log; exit 1; }
tail -1 gpurun_out/r3/chacha/t.log
for i in 1 2; do for v in A B; do
  lib=$A; [ $v = B ] && lib=$B
  PFSCDC_LIB=$lib timeout -k 10 400 python bench.py --config c4 --path commit --group 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r3/chacha/c_${v}_$i.json 2> gpurun_out/r3/chacha/c_${v}_$i.err || { tail -5 gpurun_out/r3/chacha/c_${v}_$i.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r3/chacha/c_${v}_$i.json').read().strip().splitlines()[-1]); k=d['kernel_ms']; print('$v $i', d['value'], d['ms_per_step'], round(k['create_content_hash'],2), round(k['create_ref_id'],2), d['commit_chunks_digest'])"
done; done
