#!/bin/bash
# The host-fed writer's stages with the upload split out (mirror uploads landed vs the GPU
# work after them), and the c4 commit data plane's two-set timeline (PFSCDC_TRACE).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/${1:-r5uw}
mkdir -p $o
timeout -k 10 300 python bench.py --path uw --config c4 --uw-bytes 34359738368 --steps 2 --warmup 1 > $o/uw_c4_32g.json 2> $o/uw_c4_32g.err &&
PFSCDC_TRACE=1 timeout -k 10 300 python bench.py --path commit --config c4 --group 2 --steps 3 --warmup 1 --no-cpu-baseline > $o/commit_c4_g2.json 2> $o/commit_c4_g2.err &&
timeout -k 10 300 python bench.py --path commit --config c4 --group 2 --steps 3 --warmup 1 > $o/commit_c4_g2_parity.json 2> $o/commit_c4_g2_parity.err &&
python - $o <<'PY'
import json, sys
o = sys.argv[1]
d = json.loads(open(o + "/uw_c4_32g.json").read().strip().splitlines()[-1])
print("uw", d["value"], d["ms_per_step"], d["stages_ms"], d.get("commit_filesets_digest"))
for f in ("commit_c4_g2", "commit_c4_g2_parity"):
    d = json.loads(open(o + "/%s.json" % f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["kernel_ms"], d.get("commit_chunks_digest"), d.get("parity"))
PY
