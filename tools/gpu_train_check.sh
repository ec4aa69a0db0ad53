#!/bin/bash
# One GPU session for the training path: NS=1 and NS=3 step benchmarks, then the
# kernel-trace profile of the NS=1 step (tools/profile_train.sh).  Stops at the first
# failure; each GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-r1z}
echo "== bench_train NS=1"; date
timeout -k 10 300 python scripts/bench_train.py --steps 10 --warmup 3 > gpurun_out/bench_train.log 2>&1
rc=$?; echo "rc=$rc"; tail -2 gpurun_out/bench_train.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
echo "== bench_train NS=3"; date
timeout -k 10 300 python scripts/bench_train.py --steps 5 --warmup 2 --views 3 > gpurun_out/bench_train_v3.log 2>&1
rc=$?; echo "rc=$rc"; tail -2 gpurun_out/bench_train_v3.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
echo "== profile"; date
bash tools/profile_train.sh $TAG
