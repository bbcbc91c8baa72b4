#!/bin/bash
# c4 commit G=2: issue priority of the long set (its hash launches / its ChaCha20 pass) at
# the default 30% split and at 40%; digests must not change.
set -o pipefail
cd "$(dirname "$0")/.."
o=gpurun_out/${1:-r4cs2}
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
run base &&
run nochachaprio PFSCDC_COMMIT_CHACHA_PRIO=0 &&
run nolongprio PFSCDC_COMMIT_LONG_PRIO=0 &&
run noprio PFSCDC_COMMIT_LONG_PRIO=0 PFSCDC_COMMIT_CHACHA_PRIO=0 &&
run p40_nochachaprio PFSCDC_COMMIT_LONG_PCT=40 PFSCDC_COMMIT_CHACHA_PRIO=0 &&
run p20_nochachaprio PFSCDC_COMMIT_LONG_PCT=20 PFSCDC_COMMIT_CHACHA_PRIO=0 &&
run noprio_s2 PFSCDC_COMMIT_LONG_PRIO=0 PFSCDC_COMMIT_CHACHA_PRIO=0 PFSCDC_COMMIT_SHORT_WAVES=2 &&
run base_again
