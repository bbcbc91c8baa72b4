#!/bin/bash
# c4 commit data plane: Ref.Id pass on one stream vs two (PFSCDC_REFID_TWOSTREAM), with tests.
timeout -k 10 300 python -u -m pytest tests/test_gpu_commit.py tests/test_gpu_refid.py tests/test_gpu_fileset.py tests/test_gpu_writer.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_c.log 2>&1; tail -2 gpurun_out/t_c.log
for v in 0 1 0 1; do
  PFSCDC_REFID_TWOSTREAM=$v timeout -k 10 300 python bench.py --path commit --config c4 --steps 3 --warmup 1 --no-e2e > gpurun_out/cc_$v.json 2>gpurun_out/cc_$v.err || { tail -3 gpurun_out/cc_$v.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/cc_$v.json').read().strip().splitlines()[-1]); print('two=$v', d['value'], d['ms_per_step'], d['kernel_ms']['create_content_hash'], d['kernel_ms']['create_ref_id'], d['commit_chunks_digest'], d['dataref_hashes_digest'], d.get('parity'))"
done
