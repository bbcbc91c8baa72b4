#!/bin/bash
# round 3: host-fed writer after the copy-pool split change: GPU suite, c4 8 GiB / 32 GiB / r2 workload
mkdir -p gpurun_out/r3
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3/t_gpu.log 2>&1 || { tail -30 gpurun_out/r3/t_gpu.log; exit 1; }
tail -1 gpurun_out/r3/t_gpu.log
run() {  # name args...
  name=$1; shift
  timeout -k 10 300 python bench.py --config c4 --path uw --steps 3 --warmup 1 "$@" > gpurun_out/r3/uw_$name.json 2> gpurun_out/r3/uw_$name.err || { tail -5 gpurun_out/r3/uw_$name.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r3/uw_$name.json').read().strip().splitlines()[-1]); print('$name', d['value'], d['ms_per_step'], d['commit_filesets_digest'], d.get('put_copy_gb_s'), d.get('host_memcpy_gb_s'), d['stages_ms'])"
}
run final_8g
run final_32g --uw-bytes 34359738368
run final_r2cfg --uw-bytes 6000000000
