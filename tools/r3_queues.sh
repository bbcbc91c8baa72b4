#!/bin/bash
# round 3: hardware queues (GPU_MAX_HW_QUEUES, HIP's default 4 per process): streams beyond
# them share a queue and serialize.  c3 with 2 / 4 streams in flight and the host-fed writer
# with 1 / 2 group writers, at 4 and 8 queues.
mkdir -p gpurun_out/r3q
o=gpurun_out/r3q
B="--no-cpu-baseline --no-e2e --no-literal --no-pipelined --no-chain-floor"
for Q in 4 8; do
  for K in 2 4; do
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python bench.py --config c3 --inflight $K --steps 4 --warmup 1 $B > $o/c3_q${Q}_k$K.json 2> $o/c3_q${Q}_k$K.err || { tail -5 $o/c3_q${Q}_k$K.err; exit 1; }
    python -c "
import json; d=json.loads(open('$o/c3_q${Q}_k$K.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('c3 Q=$Q K=$K', d['value'], d['ms_per_step'], round(k['hash'],1), d.get('segments_digest'), d.get('index_digest'))"
  done
  for W in 1 2; do
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 400 python bench.py --path uw --config c4 --uw-workers $W --steps 2 --warmup 1 --no-cpu-baseline > $o/uw_q${Q}_w$W.json 2> $o/uw_q${Q}_w$W.err || { tail -5 $o/uw_q${Q}_w$W.err; exit 1; }
    python -c "
import json; d=json.loads(open('$o/uw_q${Q}_w$W.json').read().strip().splitlines()[-1])
print('uw Q=$Q W=$W', d['value'], d['ms_per_step'], {k: round(v,1) for k, v in d.get('stages_ms',{}).items()}, d.get('filesets_digest'))"
  done
done
