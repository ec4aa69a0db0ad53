#!/bin/bash
# training path checks: GPU training tests, then the training step at NS = 1 and NS = 3
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -m gpu -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/train_tests.log 2>&1
rc=$?; tail -3 gpurun_out/train_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 3; do
  timeout -k 10 300 python scripts/bench_train.py --views $v --steps 10 --warmup 3 2>&1 | tail -1 | cut -c1-400 || exit $?
done
