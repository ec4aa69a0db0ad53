#!/bin/bash
# fused-epilogue cycle stamps (build the variant first: scripts/build_variant.sh epi WORKTREE
# -DPNR_EPI_TIMING) and phase timing (pt: -DPNR_PHASE_TIMING) for the three march modes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for f in 1 2 0; do
  PNR_FUSED=$f PNR_LIB_PATH=pixel-nerf_amd/build/epi/libpnr.so N_CHUNKS=10 timeout -k 10 120 python tools/mlp_probe.py || exit $?
  PNR_FUSED=$f PNR_LIB_PATH=pixel-nerf_amd/build/pt/libpnr.so N_CHUNKS=10 timeout -k 10 120 python tools/mlp_probe.py || exit $?
done
