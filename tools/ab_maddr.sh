# hoisted LDS message addresses: GPU parity of the hash paths, then the headline bench and c4
mkdir -p gpurun_out/maddr && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_refid.py tests/test_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/maddr/t.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-e2e > gpurun_out/maddr/c2.json 2> gpurun_out/maddr/c2.err && \
timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --no-e2e --no-cpu-baseline > gpurun_out/maddr/c4.json 2> gpurun_out/maddr/c4.err && \
timeout -k 10 300 python bench.py --ref-ids --steps 5 --warmup 2 --no-e2e --no-cpu-baseline > gpurun_out/maddr/c2_ref.json 2> gpurun_out/maddr/c2_ref.err
rc=$?
tail -2 gpurun_out/maddr/t.log
for f in gpurun_out/maddr/*.json; do python -c "
import json
d=json.load(open('$f')); print('$f', d['value'], d['kernel_ms'], d.get('parity'))"; done
exit $rc
