#!/bin/bash
# round 3: GPU suite, the c2 line with in-kernel clocks, c4 every-BLAKE2b line and commit data plane
mkdir -p gpurun_out/r3
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3/t_gpu.log 2>&1 || { tail -30 gpurun_out/r3/t_gpu.log; exit 1; }
tail -1 gpurun_out/r3/t_gpu.log
N="--no-e2e --no-cpu-baseline --no-literal --no-pipelined"
timeout -k 10 300 python bench.py --steps 6 --warmup 2 $N > gpurun_out/r3/c2.json 2> gpurun_out/r3/c2.err || { tail -5 gpurun_out/r3/c2.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r3/c2.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('c2', d['value'], k['scan'], k['hash'], k.get('scan_mhz'), k.get('hash_mhz'), json.dumps(d.get('roofline_valu')))"
timeout -k 10 400 python bench.py --config c4 --path commit --no-create --steps 3 --warmup 1 > gpurun_out/r3/c4_hashes.json 2> gpurun_out/r3/c4_hashes.err || { tail -5 gpurun_out/r3/c4_hashes.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r3/c4_hashes.json').read().strip().splitlines()[-1]); print('c4 hashes', d['value'], d['ms_per_step'], d['kernel_ms'], d.get('parity'), d['commit_chunks_digest'], d['dataref_hashes_digest'])"
timeout -k 10 400 python bench.py --config c4 --path commit --steps 3 --warmup 1 > gpurun_out/r3/c4_commit.json 2> gpurun_out/r3/c4_commit.err || { tail -5 gpurun_out/r3/c4_commit.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r3/c4_commit.json').read().strip().splitlines()[-1]); print('c4 commit', d['value'], d['ms_per_step'], d['kernel_ms'], d.get('parity'), d['commit_chunks_digest'], d['dataref_hashes_digest'])"
