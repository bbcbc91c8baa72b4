#!/bin/bash
# round 3: hash bins (a quad hashes a whole <= 4 MiB file) + fair-share issue priority on the
# c2 line, A/B against PFSCDC_HASH_BINS=0 / PFSCDC_HASH_FAIR=0, same box, alternating;
# parity tests first
mkdir -p gpurun_out/r3bins
o=gpurun_out/r3bins
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $o/t_parity.log 2>&1 || { tail -30 $o/t_parity.log; exit 1; }
tail -1 $o/t_parity.log
B="--no-cpu-baseline --no-e2e --no-literal --no-pipelined --no-chain-floor"
for r in 1 2; do
for cfg in "0 0" "1 0" "1 1"; do
  set -- $cfg
  PFSCDC_HASH_BINS=$1 PFSCDC_HASH_FAIR=$2 timeout -k 10 300 python bench.py --steps 10 --warmup 3 $B > $o/c2_b$1f$2_$r.json 2> $o/c2_b$1f$2_$r.err || { tail -5 $o/c2_b$1f$2_$r.err; exit 1; }
  python -c "
import json; d=json.loads(open('$o/c2_b$1f$2_$r.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('bins=$1 fair=$2 run $r', d['value'], d['ms_per_step'], round(k['scan'],2), round(k['hash'],2), round(k['hash_span'],2), round(k['hash_mhz']), d['roofline']['frac'])"
done
done
rm -f /tmp/wt.bin; PFSCDC_WAVE_TRACE=/tmp/wt.bin timeout -k 10 200 python bench.py --steps 1 --warmup 1 $B > $o/wt_bench.json 2>&1 && python tools/wave_trace.py /tmp/wt.bin > $o/wt_fair.txt; cat $o/wt_fair.txt
