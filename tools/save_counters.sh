#!/bin/bash
# Counter passes over tools/save_counters_probe.py (training forward with / without the save).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
REPO=$(pwd)
OUT=$REPO/gpurun_out/save_ctr
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum" \
           "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/g$i -o run -- python3 $REPO/tools/save_counters_probe.py > $OUT/g$i.log 2>&1
  rc=$?; echo "group $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/g$i.log; exit $rc; }
done
python3 $REPO/tools/save_counters.py $OUT/g1 $OUT/g2 $OUT/g3 $OUT/g4 | tee $OUT/summary.txt
