# Steps-in-flight overlap check over warmup/step patterns
# (with or without a second-priority stream / pacing, per the build under test)
mkdir -p gpurun_out/abi
for prio in 0; do
  for a in "c2 3 1" "c2 6 3" "c4 2 1" "c2 10 3" "c2 4 2" "c3 2 1"; do
    set -- $a
    timeout -k 10 300 python bench.py --config $1 --steps $2 --warmup $3 --no-e2e --no-cpu-baseline > gpurun_out/abi/p${prio}_$1_s$2_w$3.json 2>gpurun_out/abi/err.log || exit 1
  done
done
for f in gpurun_out/abi/*.json; do python -c "
import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['kernel_ms']['scan'], d['kernel_ms']['hash'])"; done
