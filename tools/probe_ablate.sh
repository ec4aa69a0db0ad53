#!/bin/bash
# Ablation variants of the fused MLP (built by scripts/build_variant.sh), projected-latent path.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for t in ${VARIANTS:-default gemmonly nowstream nogather}; do
  lib=pixel-nerf_amd/build/$t/libpnr.so
  [ "$t" = default ] && lib=pixel-nerf_amd/pnr/libpnr.so
  timeout -k 10 180 env PNR_LIB_PATH=$lib LATENT_PROJ=${LATENT_PROJ:-1} N_CHUNKS=10 python tools/mlp_probe.py || exit $?
done
