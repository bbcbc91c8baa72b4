#!/bin/bash
# Round 4, third GPU session: host-fed writer sweep (group writers x group size x hash issue
# priority) with the grouped index close, and a kernel trace of the c4 G=2 commit data plane
# (which launches overlap, where the GPU idles).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r4s3
bash tools/r4_uw_sweep.sh r4uw &&
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r4s3/commit_kt -o run --output-format csv -- python3 bench.py --path commit --config c4 --group 2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r4s3/commit_kt.json 2> gpurun_out/r4s3/commit_kt.err &&
ls -R gpurun_out/r4s3/commit_kt | head -20
