#!/bin/bash
# fused-march parity test against diagnostic variants (PNR_LIB_PATH), each twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for t in ${VARIANTS:-default}; do
  lib=pixel-nerf_amd/build/$t/libpnr.so; [ "$t" = default ] && lib=pixel-nerf_amd/pnr/libpnr.so
  for rep in 1 2; do
    echo -n "== $t: "
    PNR_LIB_PATH=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider \
      --timeout 120 --timeout-method thread -k "${PYTEST_K:-fused_march}" -rf 2>&1 | grep -E "passed|failed|^FAILED" | cut -c1-150 | tr '\n' ' '
    echo
  done
done
