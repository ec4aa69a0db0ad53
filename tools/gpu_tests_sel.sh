#!/bin/bash
# selected GPU tests without -x (PYTEST_K selects)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "${PYTEST_K}" > gpurun_out/sel_tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/sel_tests.log | tail -40; exit $rc
