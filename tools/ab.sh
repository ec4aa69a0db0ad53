#!/bin/bash
# A/B timing of libpnr.so variants on one box: alternates the variants (twice) through
# tools/mlp_probe.py.  Usage: tools/ab.sh tagA tagB ...  (built by build_variant.sh)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for round in 1 2; do
  for t in "$@"; do
    lib=pixel-nerf_amd/build/$t/libpnr.so
    [ "$t" = default ] && lib=pixel-nerf_amd/pnr/libpnr.so
    timeout -k 10 180 env PNR_LIB_PATH=$lib N_CHUNKS=${N_CHUNKS:-10} COMPOSITE=${COMPOSITE:-} \
      PREC=${PREC:-f16x3} python tools/mlp_probe.py || exit $?
  done
done
