# commit data plane with 1/2/3 steps in flight (c2, then c4 at 2)
mkdir -p gpurun_out/cif && \
timeout -k 10 300 python bench.py --path commit --steps 6 --warmup 1 --inflight 1 --no-e2e --no-cpu-baseline > gpurun_out/cif/c2_s1.json 2> gpurun_out/cif/c2_s1.err && \
timeout -k 10 300 python bench.py --path commit --steps 6 --warmup 1 --inflight 2 --no-e2e > gpurun_out/cif/c2_s2.json 2> gpurun_out/cif/c2_s2.err && \
timeout -k 10 300 python bench.py --path commit --steps 6 --warmup 1 --inflight 3 --no-e2e --no-cpu-baseline > gpurun_out/cif/c2_s3.json 2> gpurun_out/cif/c2_s3.err && \
timeout -k 10 300 python bench.py --path commit --config c4 --steps 4 --warmup 1 --inflight 1 --no-e2e --no-cpu-baseline > gpurun_out/cif/c4_s1.json 2> gpurun_out/cif/c4_s1.err && \
timeout -k 10 300 python bench.py --path commit --config c4 --steps 4 --warmup 1 --inflight 2 --no-e2e --no-cpu-baseline > gpurun_out/cif/c4_s2.json 2> gpurun_out/cif/c4_s2.err
rc=$?
for f in gpurun_out/cif/*.json; do python -c "
import json,sys
d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['kernel_ms'], d.get('parity'))" ; done
exit $rc
