#!/bin/bash
# c4 commit data plane at G=2 (two 100 GiB commits per step): the two-set split point and the
# waves per SIMD of each set.  Each line: value, ms/step, stage ms, digests (must not change).
set -o pipefail
cd "$(dirname "$0")/.."
o=gpurun_out/${1:-r4cs}
mkdir -p $o
run() {
  name=$1; shift
  env PFSCDC_TRACE=1 "$@" timeout -k 10 300 python bench.py --path commit --config c4 --group 2 --steps 3 --warmup 1 --no-cpu-baseline > $o/$name.json 2> $o/$name.err || return 1
  python - $o/$name.json "$name $*" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernel_ms"]
print(sys.argv[2], d["value"], d["ms_per_step"], "hash", round(k["create_content_hash"], 1), "refid", round(k["create_ref_id"], 1), d["commit_chunks_digest"], d["dataref_hashes_digest"])
PY
  grep "two sets" $o/$name.err | tail -1
}
for pct in 30 50 65 80; do
  for sw in 1 2; do
    run p${pct}_s${sw} PFSCDC_COMMIT_LONG_PCT=$pct PFSCDC_COMMIT_SHORT_WAVES=$sw || exit 1
  done
done
run p65_s2_l1 PFSCDC_COMMIT_LONG_PCT=65 PFSCDC_COMMIT_SHORT_WAVES=2 PFSCDC_COMMIT_LONG_WAVES=1 PFSCDC_COMMIT_LONG_CREATE_WAVES=1 &&
run p50_s2_l1 PFSCDC_COMMIT_LONG_PCT=50 PFSCDC_COMMIT_SHORT_WAVES=2 PFSCDC_COMMIT_LONG_WAVES=1 PFSCDC_COMMIT_LONG_CREATE_WAVES=1
