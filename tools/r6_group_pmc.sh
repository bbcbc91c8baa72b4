#!/bin/bash
# Round 6: the device group's bench line at 1/2/4/8 contexts on the one GPU, and one PMC pass
# over the scan at all CUs and at half of them (tools/scan_clock.py, 128 GiB steps).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/${1:-r6grp}
mkdir -p $o
for m in 0 0,0 0,0,0,0 0,0,0,0,0,0,0,0; do
  n=$(echo $m | tr ',' '\n' | wc -l)
  timeout -k 10 300 python bench.py --path group --members $m --steps 5 --warmup 2 > $o/group_m$n.json 2> $o/group_m$n.err || exit $?
  python -c "import json; d=json.load(open('$o/group_m$n.json')); print($n, d['value'], d['one_context']['value'], d['gather_ms'], d['gather_bytes'], d['parity'])"
done
timeout -s KILL 300 rocprofv3 --kernel-include-regex "blake2b|cdc_scan" --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_LDS_IDX_ACTIVE FETCH_SIZE -d $o/pmc -o p --output-format csv -- python3 tools/scan_clock.py 2 32768 0,128 > $o/pmc.log 2>&1 &&
python tools/pmc_per_kernel.py $o/pmc > $o/pmc_summary.txt && cat $o/pmc.log | grep scan_mhz && cat $o/pmc_summary.txt
