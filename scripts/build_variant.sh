#!/bin/bash
# Build an A/B variant of libpnr.so into pixel-nerf_amd/build/<tag>/libpnr.so.
#   [PATCH=tools/patches/<variant>.diff] scripts/build_variant.sh <tag> <git-rev|WORKTREE> [extra hipcc flags...]
# The csrc/ sources come from <rev> (or the working tree), with PATCH (a rejected schedule variant,
# tools/patches/) applied to the copy; the flags select diagnostics (csrc/pnr_diag.h) or the
# patch's knob.  Select the variant at run time with PNR_LIB_PATH=pixel-nerf_amd/build/<tag>/libpnr.so
# (diagnostic only).
set -euo pipefail
tag=$1; rev=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/pixel-nerf_amd/build/$tag
src=$out/src
rm -rf "$out"; mkdir -p "$src/csrc" "$src/include"
for f in march.hip mlp.hip train.hip encoder.hip bn.hip wgrad.hip proj.hip abi.cpp pnr_common.h march_dev.h pnr_diag.h; do
  if [ "$rev" = WORKTREE ]; then if [ -f "$root/pixel-nerf_amd/csrc/$f" ]; then cp "$root/pixel-nerf_amd/csrc/$f" "$src/csrc/$f"; fi
  else git -C "$root" show "$rev:pixel-nerf_amd/csrc/$f" > "$src/csrc/$f" 2>/dev/null || rm -f "$src/csrc/$f"; fi
done
if [ "$rev" = WORKTREE ]; then cp "$root/include/pnr_abi.h" "$src/include/"
else git -C "$root" show "$rev:include/pnr_abi.h" > "$src/include/pnr_abi.h"; fi
if [ -n "${PATCH:-}" ]; then
  case $PATCH in /*) pf=$PATCH ;; *) pf=$root/$PATCH ;; esac
  patch -s -p2 -d "$src" -i "$pf"
fi
# sources include "../../include/pnr_abi.h" relative to csrc/
mkdir -p "$out/include"; cp "$src/include/pnr_abi.h" "$out/include/"
objs=()
for f in march.hip mlp.hip train.hip encoder.hip bn.hip wgrad.hip proj.hip abi.cpp; do
  [ -f "$src/csrc/$f" ] || continue   # older revisions lack later files
  mkdir -p "$out/tmp_$f"
  # -save-temps=obj: the device assembly for isa_lint.py (the Makefile's check)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -w "$@" -I"$src/csrc" -save-temps=obj \
    -x hip -c "$src/csrc/$f" -o "$out/tmp_$f/$f.o" &
  objs+=("$out/$f.o")
done
wait
for f in march.hip mlp.hip train.hip encoder.hip bn.hip wgrad.hip proj.hip abi.cpp; do
  [ -f "$src/csrc/$f" ] || continue
  mv "$out/tmp_$f/$f.o" "$out/$f.o"
  mv "$out/tmp_$f/"*-hip-amdgcn-amd-amdhsa-gfx950.s "$out/$f.gfx950.s"
  rm -rf "$out/tmp_$f"
done
# a variant that would hand stale scratch to masked lanes never reaches the GPU (LINT=0: only to
# reproduce the round-5 fault deliberately)
if [ "${LINT:-1}" != 0 ]; then python3 "$root/pixel-nerf_amd/isa_lint.py" "$out"/*.gfx950.s; fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out/libpnr.so" "${objs[@]}" -Wl,-soname,libpnr.so \
  -Wl,-rpath,/opt/rocm/lib
echo "built $out/libpnr.so"
