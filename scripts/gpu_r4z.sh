#!/bin/bash
# Round-4 session z: the head's W_out cached in LDS -- parity / training tests, then bench_ab vs HEAD.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py tests/test_gpu_fallback.py -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/tests_r4z.log 2>&1; rc=$?
tail -2 gpurun_out/tests_r4z.log; [ $rc = 0 ] || exit $rc
VARIANTS="head default" ROUNDS=3 bash tools/bench_ab.sh 2>&1 | tee gpurun_out/ab_r4z.txt
