#!/bin/bash
# rocprofv3 kernel-trace stats of a short bench run of the headline cfg3 leg alone + separate
# PMC passes (FETCH_SIZE / WRITE_SIZE) of the headline cfg3 leg alone (one step).  Output
# under gpurun_out/prof_<tag>/; scripts/summarize_profile.py <tag> writes profiles/<tag>/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
REPO=$(pwd)
TAG=${1:-r1}
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
echo "== kernel trace"; date
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 $REPO/bench.py --steps 3 --warmup 1 --no-cpu --no-compare --no-extra --no-train --no-cfg2 \
    --no-composite > $OUT/trace_bench.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -3 $OUT/trace_bench.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
for ctr in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $ctr"; date
  timeout -k 10 600 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_$ctr -o run -- \
      python3 $REPO/bench.py --steps 1 --warmup 0 --no-cpu --no-compare --no-extra --no-train --no-cfg2 \
      --no-composite > $OUT/pmc_$ctr.log 2>&1
  rc=$?; echo "pmc $ctr rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
du -sh $OUT; find $OUT -name "*.csv" -size +20M -print -delete
