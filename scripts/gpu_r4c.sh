#!/bin/bash
# Round-4 session c: where the relu publish's split time goes.  Phase-timing
# builds (csrc/pnr_diag.h) of the cfg2 probe, wave 0 and wave 4 (the two waves of SIMD 0), and on
# wave 4 the ablations of the split VALU, the image stores and the column-maximum reads.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in pt0:0 pt4:4 pt4ns:4 pt4nst:4 pt4nc:4; do
  t=${v%%:*}; w=${v#*:}
  echo "== $t (wave $w)"
  PNR_LIB_PATH=pixel-nerf_amd/build/$t/libpnr.so PNR_FUSED=2 N_CHUNKS=8 PT_WAVE=$w \
      timeout -k 10 240 python tools/mlp_probe.py 2>&1 | grep -v amdgpu.ids || exit $?
done
