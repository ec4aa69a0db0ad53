#!/bin/bash
# Per-XCD lockstep pacing A/B: FETCH_SIZE (HBM/MALL bytes) and clock of the
# cfg3 fine-pass launches per variant, then the alternating render A/B of tools/bench_ab.sh.
# Build first (CPU): PATCH=tools/patches/lockstep.diff scripts/build_variant.sh lock1 WORKTREE -DPNR_LOCKSTEP=1
# (and lock4: =4)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
REPO=$(pwd)
export TMPDIR=/tmp
for t in ${LOCK_VARIANTS:-default lock1 lock4}; do
  lib=$REPO/pixel-nerf_amd/build/$t/libpnr.so
  [ "$t" = default ] && lib=$REPO/pixel-nerf_amd/pnr/libpnr.so
  out=$REPO/gpurun_out/lock_$t
  rm -rf $out; mkdir -p $out
  (cd /tmp && PNR_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv \
      -d $out -o run -- python3 $REPO/bench.py --steps 1 --warmup 0 --no-cpu --no-compare --no-extra --no-train \
      --no-cfg2 --no-composite > $out/bench.log 2>&1) || { echo "pmc $t failed"; tail -5 $out/bench.log; exit 1; }
  f=$(find $out -name run_counter_collection.csv | head -1)
  echo -n "$t: "; python tools/pmc_fine.py $(dirname $f) fine
  find $out -name "*.csv" -size +20M -delete
done
VARIANTS="${LOCK_VARIANTS:-default lock1 lock4}" STEPS=5 bash tools/bench_ab.sh
