N="--steps 8 --warmup 2 --no-e2e --no-cpu-baseline --no-literal --no-pipelined --no-chain-floor"
for i in 1 2; do
PFSCDC_LIB=ab/libA.so timeout -k 10 200 python bench.py $N --host-ahead 0 > gpurun_out/ab3_A_$i.json 2>/dev/null || exit 1
PFSCDC_LIB=ab/libB.so timeout -k 10 200 python bench.py $N --host-ahead 0 > gpurun_out/ab3_B0_$i.json 2>/dev/null || exit 1
PFSCDC_LIB=ab/libB.so timeout -k 10 200 python bench.py $N > gpurun_out/ab3_B1_$i.json 2>/dev/null || exit 1
for v in A B0 B1; do python -c "
import json
d=json.load(open('gpurun_out/ab3_${v}_$i.json')); k=d['kernel_ms']; print('$v', d['value'], d['ms_per_step'], round(k['scan'],2), round(k['select'],3), round(k['hash'],2), round(k['total'],2), flush=True)"; done
done
