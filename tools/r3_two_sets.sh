#!/bin/bash
# round 3: commit in two chunk sets (PFSCDC_COMMIT_TWO_SETS / _LONG_PCT / _SHORT_WAVES) against
# the one-pass form, c4 commit at G=2 (in place) and G=1; GPU commit tests first
mkdir -p gpurun_out/r3ts
o=gpurun_out/r3ts
timeout -k 10 300 python -u -m pytest tests/test_gpu_commit.py -x -q --timeout 200 --timeout-method thread > $o/t_commit.log 2>&1 || { tail -30 $o/t_commit.log; exit 1; }
tail -1 $o/t_commit.log
run() {  # name G two_sets pct short_waves [extra]
  PFSCDC_COMMIT_TWO_SETS=$3 PFSCDC_COMMIT_LONG_PCT=$4 PFSCDC_COMMIT_SHORT_WAVES=$5 timeout -k 10 400 python bench.py --config c4 --path commit --group $2 --steps 3 --warmup 1 $6 > $o/$1.json 2> $o/$1.err || { tail -5 $o/$1.err; exit 1; }
  python -c "
import json; d=json.loads(open('$o/$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('$1', d['value'], d['ms_per_step'], round(k['scan'],1), round(k['create_content_hash'],1), round(k['create'],1), d.get('parity',{}).get('ref_ids_equal_oracle'), d['commit_chunks_digest'], d['dataref_hashes_digest'])"
}
run ${P}g2_one 2 0 50 1 --no-cpu-baseline
run ${P}g2_ts50 2 1 50 1 --no-cpu-baseline
run ${P}g2_ts35 2 1 35 1 --no-cpu-baseline
run ${P}g2_ts50w2 2 1 50 2 --no-cpu-baseline
run ${P}g1_one 1 0 50 1 --no-cpu-baseline
run ${P}g1_ts50 1 1 50 1
for Q in 8 16; do
for K in 4 8; do
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python bench.py --config c3 --inflight $K --steps 4 --warmup 1 --no-cpu-baseline --no-e2e --no-literal --no-pipelined --no-chain-floor > $o/c3_q${Q}_k$K.json 2> $o/c3_q${Q}_k$K.err || { tail -5 $o/c3_q${Q}_k$K.err; exit 1; }
  python -c "
import json; d=json.loads(open('$o/c3_q${Q}_k$K.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('c3 Q=$Q K=$K', d['value'], d['ms_per_step'], round(k['hash'],1), round(k['hash_span'],1), d.get('parity'))"
done
done
