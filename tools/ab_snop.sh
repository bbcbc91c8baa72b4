#!/bin/bash
timeout -k 10 300 env PFSCDC_LIB=ab/libB.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_refid.py tests/test_gpu_commit.py tests/test_gpu_rechunk.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -1
bash tools/ab_lib2.sh ab/libA.so ab/libB.so 2
