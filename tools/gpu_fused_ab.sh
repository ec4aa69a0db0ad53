#!/bin/bash
# fused ray march: GPU parity tests, then an A/B (tools/bench_ab.sh variants) of full fusion,
# fusion without the fine draws, separate kernels, the non-deferred epilogue (nodefer) and
# the previous revision's build (head)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    ${PYTEST_ARGS} > gpurun_out/fused_tests.log 2>&1
rc=$?; tail -5 gpurun_out/fused_tests.log; [ $rc -eq 0 ] || exit $rc
VARIANTS=${VARIANTS:-"default default:--fused-mode=2 default:--unfused nodefer head"} STEPS=5 timeout -k 10 900 bash tools/bench_ab.sh
