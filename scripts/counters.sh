#!/bin/bash
# PMC passes over a probe script (default tools/mlp_probe.py; one rocprofv3 run per
# counter group).  Usage: counters.sh <tag> [probe.py]
# EXTRA_GROUPS=1 adds a FETCH_SIZE pass (HBM/MALL bytes; 3 of the 4 TCC counters).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
REPO=$(pwd)
OUT=$REPO/gpurun_out/ctr_${1:-x}
PROBE=$REPO/${2:-tools/mlp_probe.py}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum" \
           ${EXTRA_GROUPS:+"FETCH_SIZE"}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/g$i -o run -- python3 $PROBE > $OUT/g$i.log 2>&1
  rc=$?; echo "group $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/g$i.log; exit $rc; }
done
