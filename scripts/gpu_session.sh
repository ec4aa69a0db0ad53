#!/bin/bash
# One parameterized GPU session (replaces the per-session scripts of round 4).
#   scripts/gpu_session.sh <tag> <step> [<step> ...]
# Steps (run in the order given; the session stops at the first failing step):
#   tests      pytest -m gpu (PYTEST_ARGS adds selectors / -k)            -> gpurun_out/<tag>/gpu_tests.log
#   smoke      __graft_entry__.smoke()                                     -> gpurun_out/<tag>/smoke.log
#   evidence   the same-lease roofline evidence, in this order:
#                PMC passes FETCH_SIZE, WRITE_SIZE, GRBM_GUI_ACTIVE over the cfg3 headline leg and the
#                1 M-ray composite leg; their summary (scripts/summarize_profile.py); the full bench
#                reading that summary (--traffic-from); a kernel-trace run of the headline leg.
#              -> gpurun_out/prof_<tag>/ (summary/ holds pmc_summary.csv, clock.csv, kernel_stats.csv,
#                 mlp_dispatch_stats.csv, bench_line.json)
#   bench      the default bench line alone (BENCH_ARGS)                   -> gpurun_out/<tag>/bench.log
#   cmd:<c>    any further command (e.g. cmd:"python tools/wgrad_trajectory.py"), TIMEOUT_S each
# Every GPU step runs under its own `timeout -k 10`.  Record the session's arguments in
# profiles/<tag>/README when committing its outputs.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
REPO=$(pwd)
TAG=${1:?tag}; shift
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
PY=python3
run() {  # run <timeout_s> <log> <cmd...>
  local t=$1 log=$2; shift 2
  echo "== $(date +%T) $*"
  timeout -k 10 $t "$@" > $log 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -3 $log | cut -c1-400
  return $rc
}
for step in "$@"; do
  case "$step" in
    tests)
      run ${TIMEOUT_S:-900} $OUT/gpu_tests.log $PY -u -m pytest tests -m gpu -v -p no:cacheprovider -rA \
          --timeout 300 --timeout-method thread ${PYTEST_ARGS} || exit $? ;;
    smoke)
      run 300 $OUT/smoke.log $PY -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench)
      run 600 $OUT/bench.log $PY bench.py ${BENCH_ARGS} || exit $? ;;
    evidence)
      P=$REPO/gpurun_out/prof_$TAG
      mkdir -p $P
      LEG="--steps 1 --warmup 0 --no-cpu --no-compare --no-extra --no-train --no-cfg2 --no-clock"
      export TMPDIR=/tmp
      for ctr in FETCH_SIZE WRITE_SIZE GRBM_GUI_ACTIVE; do
        ( cd /tmp && run 300 $P/pmc_$ctr.log rocprofv3 --pmc $ctr --output-format csv -d $P/pmc_$ctr -o run -- \
            $PY $REPO/bench.py $LEG ) || exit $?
      done
      ( cd /tmp && run 300 $P/trace.log rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- \
          $PY $REPO/bench.py --steps 3 --warmup 1 --no-cpu --no-compare --no-extra --no-train --no-cfg2 \
          --no-composite ) || exit $?
      PNR_PROFILE_DST=$P/summary $PY scripts/summarize_profile.py $TAG "(same lease as bench_line.json)" \
          > $P/summarize.log 2>&1 || { cat $P/summarize.log; exit 1; }
      run 900 $P/bench.log $PY bench.py --traffic-from $P/summary/pmc_summary.csv ${BENCH_ARGS} || exit $?
      grep '^{' $P/bench.log | tail -1 > $P/summary/bench_line.json
      find $P -name "*.csv" -size +20M -delete ;;
    cmd:*)
      run ${TIMEOUT_S:-600} $OUT/cmd_$(date +%H%M%S).log bash -c "${step#cmd:}" || exit $? ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
