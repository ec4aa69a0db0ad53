#!/bin/bash
# HBM bytes per training-step kernel: rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate passes
# (the gfx950 TCC limit) of scripts/bench_train.py --steps 1 --warmup 1, summarised per kernel by
# tools/pmc_train_summary.py.  Output under gpurun_out/pmc_train_<tag>/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
REPO=$(pwd)
OUT=$REPO/gpurun_out/pmc_train_${1:-r4}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $ctr"
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d $OUT/$ctr -o run -- \
      python3 $REPO/scripts/bench_train.py --steps 1 --warmup 1 > $OUT/$ctr.log 2>&1
  rc=$?; echo "pmc $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 $REPO/tools/pmc_train_summary.py $OUT
