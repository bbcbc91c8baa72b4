#!/bin/bash
# (Historical: PFSCDC_HASH_FORK exists only with profiles/r5/rejected/first_piece_fork/
# fork.patch applied; the form was rejected and removed.)
# The first-piece fork in pfscdc_commit_refs (PFSCDC_HASH_FORK): GPU parity of the commit
# suites, then c4 commits (G = 2) with the fork on and off alternating on one box, then the
# host-fed writer's stages with the upload split out (mirror uploads landed vs GPU work).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/${1:-r5fork}
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_commit.py tests/test_gpu_fileset.py tests/test_gpu_refid.py -x -q --timeout 200 --timeout-method thread > $o/pytest_commit.log 2>&1 && tail -1 $o/pytest_commit.log || exit 1
for i in 1 2; do
  for f in 1 0; do
    PFSCDC_HASH_FORK=$f PFSCDC_TRACE=1 timeout -k 10 300 python bench.py --path commit --config c4 --group 2 --steps 3 --warmup 1 --no-cpu-baseline > $o/commit_f${f}_$i.json 2> $o/commit_f${f}_$i.err || exit 1
  done
done
timeout -k 10 300 python bench.py --path uw --config c4 --uw-bytes 34359738368 --steps 2 --warmup 1 > $o/uw_c4_32g.json 2> $o/uw_c4_32g.err || exit 1
python - $o <<'PY'
import json, sys, glob
o = sys.argv[1]
for f in sorted(glob.glob(o + "/commit_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["value"], d["ms_per_step"], {k: round(v, 1) for k, v in d["kernel_ms"].items()},
          d.get("commit_chunks_digest"), d.get("dataref_hashes_digest"))
d = json.loads(open(o + "/uw_c4_32g.json").read().strip().splitlines()[-1])
print("uw", d["value"], d["ms_per_step"], d["stages_ms"], d.get("commit_filesets_digest"))
PY
