#!/bin/bash
# bench.py (render line only) for libpnr.so variants in one box session, alternating.
# Usage: VARIANTS="tagA default" bash tools/bench_ab.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for round in 1 2; do
  for t in ${VARIANTS:-default}; do
    lib=pixel-nerf_amd/build/$t/libpnr.so
    [ "$t" = default ] && lib=pixel-nerf_amd/pnr/libpnr.so
    echo -n "$t: "
    PNR_LIB_PATH=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-extra --no-composite --no-compare 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms']['mlp_coarse'], d['kernel_ms']['mlp_fine'])" || exit $?
  done
done
