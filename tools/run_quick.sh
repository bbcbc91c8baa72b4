# gpu tests + one bench line (inflight 1 and 4)
mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/tq.log 2>&1 && \
timeout -k 10 300 python bench.py --inflight 1 --steps 10 --no-cpu-baseline --no-e2e > gpurun_out/bq1.json 2> gpurun_out/bq1.err && \
timeout -k 10 300 python bench.py --inflight 4 --steps 16 --no-cpu-baseline --no-e2e > gpurun_out/bq4.json 2> gpurun_out/bq4.err
echo rc=$?
