#!/bin/bash
# Training-path check after a change: the GPU training tests, the NS=1 step benchmark and
# its kernel-trace profile (tag $1).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-ab}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_train.py > gpurun_out/t_train_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t_train_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_train.py --steps 10 --warmup 3 > gpurun_out/bench_train_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_train_$TAG.log | cut -c1-220
[ $rc -eq 0 ] || exit $rc
bash scripts/profile_train.sh $TAG > /dev/null
rc=$?; echo "profile rc=$rc"; head -18 gpurun_out/prof_train_$TAG/step_breakdown.txt
exit $rc
