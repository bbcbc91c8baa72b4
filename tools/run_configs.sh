# gpu tests + one bench line per BASELINE config (c2 headline, c3 stream, c4 commit, c5 dedup)
mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 > gpurun_out/bc3.json 2> gpurun_out/bc3.err && \
timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 > gpurun_out/bc4.json 2> gpurun_out/bc4.err && \
timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/bc5.json 2> gpurun_out/bc5.err && \
timeout -k 10 300 python bench.py --config c5 --dedup files --steps 3 --warmup 1 > gpurun_out/bc5f.json 2> gpurun_out/bc5f.err
echo rc=$?
