#!/bin/bash
# What the training forward's activation save costs, by part (diagnostic builds, results invalid):
# tools/fwd_save_ab.py on the shipped library and on builds without the fp32 save-slot stores
# (savef: -DPNR_ABLATE_SAVEF), without the relu-mask stores (savem: -DPNR_ABLATE_SAVEM) and without
# both (savefm); scripts/build_variant.sh <name> WORKTREE <flags>.  csrc/pnr_diag.h.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for lib in ${VARIANTS:-default savef savem savefm}; do
  echo "== $lib"
  if [ $lib = default ]; then unset PNR_LIB_PATH; else export PNR_LIB_PATH=pixel-nerf_amd/build/$lib/libpnr.so; fi
  timeout -k 10 300 python tools/fwd_save_ab.py 2>/dev/null | grep round || exit 1
done
