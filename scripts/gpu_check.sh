#!/bin/bash
# One GPU session: parity tests, smoke, short bench.  Stops at the first fault /
# abort / timeout (exit codes other than 0 or 1).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
echo "== pytest -m gpu"; date
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider -rA --timeout 300 \
    --timeout-method thread ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/gpu_tests.log | tail -30
ok $rc || exit $rc
echo "== smoke"; date
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
ok $rc || exit $rc
[ -n "$NO_BENCH" ] && exit 0
echo "== bench"; date
timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-5} --warmup 1 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench.log
exit $rc
