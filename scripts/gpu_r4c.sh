#!/bin/bash
# Round-4 session c: where the relu publish's split time goes -- phase-timing
# builds (csrc/pnr_diag.h) of the cfg2 probe, wave 0 and wave 4 (the two waves of SIMD 0), and on
# wave 4 the ablations of the split VALU, the image stores and the column-maximum reads -- then the
# full bench of HEAD.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in pt0:0 pt4:4 pt4ns:4 pt4nst:4 pt4nc:4; do
  t=${v%%:*}; w=${v#*:}
  echo "== $t (wave $w)"
  PNR_LIB_PATH=pixel-nerf_amd/build/$t/libpnr.so PNR_FUSED=2 N_CHUNKS=8 PT_WAVE=$w \
      timeout -k 10 240 python tools/mlp_probe.py > gpurun_out/phase_$t.txt 2>&1 || { cat gpurun_out/phase_$t.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/phase_$t.txt
done
echo "== bench"; date
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_r4c.log 2>&1; rc=$?
tail -c 2500 gpurun_out/bench_r4c.log; exit $rc
