mkdir -p gpurun_out/cif2 && \
timeout -k 10 300 python bench.py --path commit --steps 8 --warmup 1 --inflight 4 --no-e2e --no-cpu-baseline > gpurun_out/cif2/c2_s4.json 2> gpurun_out/cif2/c2_s4.err && \
timeout -k 10 300 python bench.py --path commit --config c4 --steps 6 --warmup 1 --inflight 3 --no-e2e --no-cpu-baseline > gpurun_out/cif2/c4_s3.json 2> gpurun_out/cif2/c4_s3.err && \
timeout -k 10 300 python bench.py --path commit --config c4 --steps 8 --warmup 1 --inflight 4 --no-e2e > gpurun_out/cif2/c4_s4.json 2> gpurun_out/cif2/c4_s4.err
rc=$?
for f in gpurun_out/cif2/*.json; do python -c "
import json,sys
d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['kernel_ms'], d.get('parity'))" ; done
exit $rc
