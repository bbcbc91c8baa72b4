#!/bin/bash
# round 3: two-set commit with the long set's content chains only (PFSCDC_COMMIT_LONG_CHAINS)
# at several split points, against the one-pass form and the round's two-set form; c4 G=2
mkdir -p gpurun_out/r3ch
o=gpurun_out/r3ch
timeout -k 10 300 python -u -m pytest tests/test_gpu_commit.py -x -q --timeout 200 --timeout-method thread > $o/t_commit.log 2>&1 || { tail -30 $o/t_commit.log; exit 1; }
tail -1 $o/t_commit.log
run() {  # name two_sets chains pct
  PFSCDC_COMMIT_TWO_SETS=$2 PFSCDC_COMMIT_LONG_CHAINS=$3 PFSCDC_COMMIT_LONG_PCT=$4 timeout -k 10 400 python bench.py --config c4 --path commit --group 2 --steps 3 --warmup 1 --no-cpu-baseline > $o/$1.json 2> $o/$1.err || { tail -5 $o/$1.err; exit 1; }
  python -c "
import json; d=json.loads(open('$o/$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('$1', d['value'], d['ms_per_step'], round(k['scan'],1), round(k['create_content_hash'],1), round(k['create'],1), d['commit_chunks_digest'], d['dataref_hashes_digest'])"
}
run one 0 1 30
run ts30 1 0 30
run ch30 1 1 30
run ch50 1 1 50
run ch65 1 1 65
run ch80 1 1 80
