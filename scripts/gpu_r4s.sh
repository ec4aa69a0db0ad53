#!/bin/bash
# Round-4 session s: the fp32 VALU head from the accumulators (no last publish, no split-fp16 head
# GEMM) -- the parity / training GPU tests on it, then bench_ab against the HEAD build, alternating.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "== parity + training tests"
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py tests/test_gpu_fallback.py -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/tests_r4s.log 2>&1; rc=$?
tail -2 gpurun_out/tests_r4s.log; [ $rc = 0 ] || exit $rc
echo "== bench A/B"
VARIANTS="head default" ROUNDS=3 bash tools/bench_ab.sh 2>&1 | tee gpurun_out/ab_r4s.txt
