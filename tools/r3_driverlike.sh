#!/bin/bash
# What the driver runs at round end, on the final tree: the GPU suite, smoke(), and the
# default bench line (no flags)
mkdir -p gpurun_out/r3dl
o=gpurun_out/r3dl
timeout -k 10 420 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $o/pytest_gpu.log 2>&1 && tail -1 $o/pytest_gpu.log && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 && tail -1 $o/smoke.log && \
timeout -k 10 400 python bench.py > $o/bench.json 2> $o/bench.err && python -c "
import json; d=json.loads(open('$o/bench.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print(d['value'], d['ms_per_step'], d['steps'], d['warmup'], round(k['scan'],2), round(k['hash'],2), round(k['scan_mhz']), round(k['hash_mhz']), d['roofline']['frac'], d['roofline']['traffic'], d['parity'], d['cpu_baseline']['value'])"
