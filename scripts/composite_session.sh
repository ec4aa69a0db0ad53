# Composite A/B session (round 5): the numerical check of each library (tools/composite_check.py)
# and the alternating 1 M-ray timing (tools/composite_ab.sh).  VARIANTS names libraries under
# pixel-nerf_amd/build/<name>/ (scripts/build_variant.sh, the rejected layouts from
# tools/patches/composite_variants.diff); "default" is the tree's own.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
VARIANTS=${VARIANTS:-"default compc"}   # compc: PATCH=tools/patches/composite_variants.diff scripts/build_variant.sh compc WORKTREE
for t in $VARIANTS; do
  lib=pixel-nerf_amd/build/$t/libpnr.so; [ $t = default ] && lib=pixel-nerf_amd/pnr/libpnr.so
  echo "== check $t"; PNR_LIB_PATH=$lib timeout -k 10 120 python tools/composite_check.py 2>/dev/null | tail -12
done
VARIANTS="$VARIANTS" ROUNDS=3 timeout -k 10 300 bash tools/composite_ab.sh
