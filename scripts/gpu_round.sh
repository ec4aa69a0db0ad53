#!/bin/bash
# One GPU session for the round's evidence: GPU tests + smoke + full bench (scripts/gpu_check.sh),
# then the rocprofv3 kernel trace + PMC passes of the headline leg (scripts/profile.sh <tag>).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r2d}
BENCH_STEPS=${BENCH_STEPS:-10} bash scripts/gpu_check.sh || exit $?
cp gpurun_out/bench.log gpurun_out/bench_$TAG.log
bash scripts/profile.sh $TAG
