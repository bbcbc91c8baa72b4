#!/bin/bash
# Whole GPU suite, smoke and the default bench line (what the driver runs at round end).
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_gpu.log 2>&1; tail -1 gpurun_out/t_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
timeout -k 10 400 python bench.py > gpurun_out/bench_final.json 2>gpurun_out/bench_final.err || { tail -3 gpurun_out/bench_final.err; exit 1; }
python -c "
import json
d=json.loads(open('gpurun_out/bench_final.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'], d['parity'])"
