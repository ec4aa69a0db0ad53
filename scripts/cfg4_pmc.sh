#!/bin/bash
# FETCH_SIZE per k_point_mlp launch of the cfg4 DTU frame in input order and in the renderer's
# blocked processing order (tools/cfg4_probe.py, tools/pmc_cfg4.py).
#   bash scripts/cfg4_pmc.sh <tag>   -> gpurun_out/<tag>/pmc_cfg4.jsonl
cd "${GRAFT_REPO_ROOT:-/root/repo}"
REPO=$(pwd)
OUT=$REPO/gpurun_out/${1:?tag}
mkdir -p $OUT
export TMPDIR=/tmp
for ro in input auto; do
  ( cd /tmp && RAY_ORDER=$ro N_FRAMES=1 timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv \
      -d $OUT/pmc_cfg4_$ro -o run -- python3 $REPO/tools/cfg4_probe.py > $OUT/pmc_cfg4_$ro.log 2>&1 ) || exit $?
  python3 $REPO/tools/pmc_cfg4.py $(find $OUT/pmc_cfg4_$ro -name "*counter_collection.csv" | head -1) $ro \
      >> $OUT/pmc_cfg4.jsonl || exit $?
  find $OUT/pmc_cfg4_$ro -name "*.csv" -size +20M -delete
done
cat $OUT/pmc_cfg4.jsonl | cut -c1-400
