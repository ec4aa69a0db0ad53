#!/bin/bash
# k_points_in_bwd run length (points per wave, -DPNR_PIB_RUN) A/B: per variant one kernel-trace of
# scripts/bench_train.py (3 steps) for the kernel's own time, then the alternating training step
# (tools/train_lib_ab.sh).  Variants: default (8), run4, run16 (scripts/build_variant.sh runN WORKTREE -DPNR_PIB_RUN=N).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
REPO=$(pwd)
OUT=$REPO/gpurun_out/pib_ab
mkdir -p $OUT
export TMPDIR=/tmp
for t in ${VARIANTS:-default run4 run16}; do
  lib=$REPO/pixel-nerf_amd/build/$t/libpnr.so; [ "$t" = default ] && lib=$REPO/pixel-nerf_amd/pnr/libpnr.so
  ( cd /tmp && PNR_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$t -o run -- \
      python3 $REPO/scripts/bench_train.py --steps 3 --warmup 1 > $OUT/$t.log 2>&1 ) || exit $?
  f=$(find $OUT/$t -name "*kernel_stats.csv" | head -1)
  echo "$t: $(grep -h "k_points_in_bwd" $f | cut -d, -f2-4)"
done
VARIANTS="${VARIANTS:-default run4 run16}" bash tools/train_lib_ab.sh
