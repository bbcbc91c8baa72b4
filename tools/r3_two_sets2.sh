#!/bin/bash
# round 3: two-set commit split-point sweep (PFSCDC_COMMIT_LONG_PCT) with 4 and 8 hardware
# queues; c3 in flight with 8 queues; host-fed writer with 1 / 2 group writers at 8 queues
mkdir -p gpurun_out/r3ts2
o=gpurun_out/r3ts2
run() {  # name G two_sets pct queues [extra]
  GPU_MAX_HW_QUEUES=$5 PFSCDC_COMMIT_TWO_SETS=$3 PFSCDC_COMMIT_LONG_PCT=$4 timeout -k 10 400 python bench.py --config c4 --path commit --group $2 --steps 3 --warmup 1 --no-cpu-baseline $6 > $o/$1.json 2> $o/$1.err || { tail -5 $o/$1.err; exit 1; }
  python -c "
import json; d=json.loads(open('$o/$1.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('$1', d['value'], d['ms_per_step'], round(k['scan'],1), round(k['create_content_hash'],1), round(k['create'],1), d['commit_chunks_digest'], d['dataref_hashes_digest'])"
}
run g2_one_q4 2 0 50 4
run g2_one_q8 2 0 50 8
for pct in 10 20 30 40; do run g2_ts${pct}_q4 2 1 $pct 4; done
run g2_ts20_q8 2 1 20 8
run g2_ts30_q8 2 1 30 8
run g1_one_q8 1 0 50 8
for pct in 10 20 35; do run g1_ts${pct}_q4 1 1 $pct 4; done
