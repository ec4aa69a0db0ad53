#!/bin/bash
# Phase timing + gather ablation of the projected-latent path vs the latent-gather path.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for lp in 1 0; do
  for t in default phase nogather; do
    lib=pixel-nerf_amd/build/$t/libpnr.so
    [ "$t" = default ] && lib=pixel-nerf_amd/pnr/libpnr.so
    timeout -k 10 180 env PNR_LIB_PATH=$lib LATENT_PROJ=$lp N_CHUNKS=10 python tools/mlp_probe.py || exit $?
  done
done
