set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for t in default compc; do
  lib=pixel-nerf_amd/build/$t/libpnr.so; [ $t = default ] && lib=pixel-nerf_amd/pnr/libpnr.so
  echo "== check $t"; PNR_LIB_PATH=$lib timeout -k 10 120 python tools/composite_check.py 2>/dev/null | tail -12
done
VARIANTS="default compc" ROUNDS=3 timeout -k 10 300 bash tools/composite_ab.sh
