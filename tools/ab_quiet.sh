# parity of every hash mode with the countdown, then same-box A/B vs the previous build
mkdir -p gpurun_out/quiet && \
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/quiet/t.log 2>&1 && \
bash tools/ab_lib.sh pfs_amd/libpfscdc_old.so pfs_amd/libpfscdc.so 2 && \
timeout -k 10 300 python bench.py --ref-ids --steps 5 --warmup 2 --no-e2e --no-cpu-baseline > gpurun_out/quiet/c2_ref.json 2> gpurun_out/quiet/c2_ref.err && \
timeout -k 10 300 python bench.py --config c3 --steps 2 --warmup 1 --no-e2e --no-cpu-baseline > gpurun_out/quiet/c3.json 2> gpurun_out/quiet/c3.err
rc=$?
tail -2 gpurun_out/quiet/t.log
for f in gpurun_out/quiet/*.json; do python -c "
import json
d=json.load(open('$f')); print('$f', d['value'], d['kernel_ms'])"; done
exit $rc
