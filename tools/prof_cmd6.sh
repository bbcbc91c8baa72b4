mkdir -p gpurun_out && hipcc --offload-arch=gfx950 -O3 tools/ubench.hip -o /tmp/ubench 2>/dev/null && timeout -k 10 120 /tmp/ubench > gpurun_out/ubench2.txt 2>&1; echo rc=$?
