#!/bin/bash
# Round-4 session m: where the cfg4 (NS = 3) frame's time goes -- default vs the projected-row
# gather ablated (results invalid), and the phase-timing build's per-tile phases on cfg4 and cfg2.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for round in 1 2; do
  for t in default ablate_gather; do
    lib=pixel-nerf_amd/build/$t/libpnr.so; [ $t = default ] && lib=pixel-nerf_amd/pnr/libpnr.so
    PNR_LIB_PATH=$lib N_FRAMES=2 timeout -k 10 300 python tools/cfg4_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done | tee gpurun_out/cfg4_ab.txt
for w in 0 4; do
  PNR_PT_WAVE=$w true
done
PNR_LIB_PATH=pixel-nerf_amd/build/phase/libpnr.so N_FRAMES=1 timeout -k 10 300 python tools/cfg4_probe.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/cfg4_ab.txt
PNR_LIB_PATH=pixel-nerf_amd/build/phase/libpnr.so N_CHUNKS=8 timeout -k 10 300 python tools/mlp_probe.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/cfg4_ab.txt
