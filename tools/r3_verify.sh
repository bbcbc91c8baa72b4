#!/bin/bash
# round 3: GPU suite after the dek-count fix, and a per-XCD wave trace (clocks) of the c2 hash
mkdir -p gpurun_out/r3v
o=gpurun_out/r3v
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $o/pytest_gpu.log 2>&1 || { tail -30 $o/pytest_gpu.log; exit 1; }
tail -1 $o/pytest_gpu.log
B="--no-cpu-baseline --no-e2e --no-literal --no-pipelined --no-chain-floor"
rm -f /tmp/wt.bin; PFSCDC_WAVE_TRACE=/tmp/wt.bin timeout -k 10 200 python bench.py --steps 1 --warmup 1 $B > $o/wt_bench.json 2>&1 && python tools/wave_trace.py /tmp/wt.bin > $o/wt_xcd.txt && cat $o/wt_xcd.txt
timeout -k 10 300 python bench.py --ref-ids --steps 3 --warmup 1 $B > $o/c2_refids.json 2> $o/c2_refids.err || { tail -5 $o/c2_refids.err; exit 1; }
python -c "
import json; d=json.loads(open('$o/c2_refids.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('c2 ref-ids', d['value'], d['ms_per_step'], {a: round(b,2) for a,b in k.items() if isinstance(b,float)})"
