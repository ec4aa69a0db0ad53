#!/bin/bash
# Weight re-streaming bound: the production build against
# -DPNR_ABLATE_WSTREAM (every k-step re-reads k-step 0's fragments, L1/L2-hot: no weight
# stream, wrong results, timing only).  PMC passes of both over tools/mlp_probe.py (2 cfg2
# chunks) including FETCH_SIZE, then the alternating render A/B of tools/bench_ab.sh.
# Build first (CPU): bash scripts/build_variant.sh wsab WORKTREE -DPNR_ABLATE_WSTREAM
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for t in default wsab; do
  lib=pixel-nerf_amd/build/$t/libpnr.so
  [ "$t" = default ] && lib=pixel-nerf_amd/pnr/libpnr.so
  echo "== counters $t"
  PNR_LIB_PATH=$PWD/$lib EXTRA_GROUPS=1 bash scripts/counters.sh ws_$t || exit $?
  python scripts/analyze_counters.py gpurun_out/ctr_ws_$t | tee gpurun_out/ctr_ws_$t/summary.txt
done
VARIANTS="wsab default" STEPS=5 bash tools/bench_ab.sh
