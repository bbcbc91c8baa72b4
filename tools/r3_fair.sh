#!/bin/bash
# round 3: fair-share variants on the c2 line (same box, alternating), a per-XCD wave trace,
# and the c3 line at its new defaults (four streams in flight, 8 hardware queues)
mkdir -p gpurun_out/r3fair
o=gpurun_out/r3fair
B="--no-cpu-baseline --no-e2e --no-literal --no-pipelined --no-chain-floor"
for r in 1 2; do
for cfg in "1 1 256" "1 1 64" "0 2 256" "1 1 1024"; do
  set -- $cfg
  n=b$1f$2e$3_$r
  PFSCDC_HASH_BINS=$1 PFSCDC_HASH_FAIR=$2 PFSCDC_HASH_FAIR_EVERY=$3 timeout -k 10 300 python bench.py --steps 10 --warmup 3 $B > $o/$n.json 2> $o/$n.err || { tail -5 $o/$n.err; exit 1; }
  python -c "
import json; d=json.loads(open('$o/$n.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('$n', d['value'], d['ms_per_step'], round(k['scan'],2), round(k['hash'],2), round(k['hash_mhz']), d['roofline']['frac'])"
done
done
rm -f /tmp/wt.bin; PFSCDC_WAVE_TRACE=/tmp/wt.bin timeout -k 10 200 python bench.py --steps 1 --warmup 1 $B > $o/wt_bench.json 2>&1 && python tools/wave_trace.py /tmp/wt.bin > $o/wt_fair.txt && cat $o/wt_fair.txt
timeout -k 10 300 python bench.py --config c3 --steps 4 --warmup 1 > $o/c3.json 2> $o/c3.err || { tail -5 $o/c3.err; exit 1; }
python -c "
import json; d=json.loads(open('$o/c3.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('c3', d['value'], d['ms_per_step'], d['config'].get('steps_in_flight'), round(k['hash'],1), d.get('one_step_alone'), d.get('index_digest'), d.get('parity'))"
