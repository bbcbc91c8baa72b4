# microbenchmarks + FETCH_SIZE calibration of the memory patterns
mkdir -p gpurun_out && export TMPDIR=/tmp && \
hipcc --offload-arch=gfx950 -O3 tools/ubench.hip -o /tmp/ubench 2>/dev/null && \
timeout -k 10 120 /tmp/ubench > gpurun_out/ubench.txt 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-include-regex rd_ --pmc FETCH_SIZE -d gpurun_out/pmc5 -o p --output-format csv -- /tmp/ubench > gpurun_out/pmc5.log 2>&1 && \
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1
echo rc=$?
