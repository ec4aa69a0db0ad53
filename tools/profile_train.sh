#!/bin/bash
# rocprofv3 kernel-trace stats of the training-step benchmark (scripts/bench_train.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
REPO=$(pwd)
OUT=$REPO/gpurun_out/prof_train_${1:-r1}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
    python3 $REPO/scripts/bench_train.py --steps 3 --warmup 1 > $OUT/log.txt 2>&1
rc=$?; echo "trace rc=$rc"; tail -2 $OUT/log.txt | cut -c1-300
[ $rc -eq 0 ] || exit $rc
# keep the stats and a one-step breakdown; the raw trace is too large to copy back
python3 $REPO/tools/train_step_breakdown.py $(find $OUT -name "*kernel_trace.csv" | head -1) 40 > $OUT/step_breakdown.txt
find $OUT -name "*kernel_trace.csv" -delete
head -60 $OUT/step_breakdown.txt
