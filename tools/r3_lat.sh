#!/bin/bash
# round 3: latency form of the rounds for one-wave-per-SIMD hash launches, same-box A/B
mkdir -p gpurun_out/r3/lat
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3/t_gpu.log 2>&1 || { tail -30 gpurun_out/r3/t_gpu.log; exit 1; }
tail -1 gpurun_out/r3/t_gpu.log
for rep in 1 2; do
  for L in 0 1; do
    PFSCDC_HASH_LAT=$L timeout -k 10 120 python tools/chain_latency.py 8388608 2.4 1,4096 > gpurun_out/r3/lat/chain_L${L}_$rep.txt 2>&1 || exit 1
    grep chains gpurun_out/r3/lat/chain_L${L}_$rep.txt | sed "s/^/L=$L /"
    PFSCDC_HASH_LAT=$L timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r3/lat/c4_L${L}_$rep.json 2> gpurun_out/r3/lat/c4_L${L}_$rep.err || { tail -5 gpurun_out/r3/lat/c4_L${L}_$rep.err; exit 1; }
    PFSCDC_HASH_LAT=$L timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r3/lat/c3_L${L}_$rep.json 2> gpurun_out/r3/lat/c3_L${L}_$rep.err || { tail -5 gpurun_out/r3/lat/c3_L${L}_$rep.err; exit 1; }
    python -c "
import json
for c in ('c4','c3'):
    d=json.loads(open('gpurun_out/r3/lat/%s_L${L}_$rep.json' % c).read().strip().splitlines()[-1]); k=d['kernel_ms']
    print('L=$L', c, d['value'], d['ms_per_step'], round(k['hash'],2), round(k.get('hash_span',0),2), round(k.get('hash_mhz',0)), d.get('index_digest'))"
  done
done
bash tools/scale_predict.sh > gpurun_out/r3/scale_predict.txt 2>&1 || { tail -5 gpurun_out/r3/scale_predict.txt; exit 1; }
grep json gpurun_out/r3/scale_predict.txt
