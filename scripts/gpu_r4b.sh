#!/bin/bash
# Round-4 session b: GPU tests + smoke, render / training A/B of HEAD against the pre-prune kernel
# (build/pre), a one-step training profile, and the fine-pass PMC groups of HEAD.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
NO_BENCH=1 bash scripts/gpu_check.sh || exit $?
echo "== render A/B"; date
VARIANTS="pre default" ROUNDS=2 STEPS=5 bash tools/bench_ab.sh > gpurun_out/ab_r4b.txt 2>&1; rc=$?
cat gpurun_out/ab_r4b.txt; [ $rc -eq 0 ] || exit $rc
echo "== train A/B"; date
VARIANTS="pre default" STEPS=20 bash tools/train_lib_ab.sh > gpurun_out/ab_r4b_train.txt 2>&1; rc=$?
cat gpurun_out/ab_r4b_train.txt; [ $rc -eq 0 ] || exit $rc
echo "== train profile"; date
bash tools/profile_train.sh r4b || exit $?
echo "== counters"; date
PNR_FUSED=2 N_CHUNKS=4 bash scripts/counters.sh r4b || exit $?
python3 scripts/analyze_counters.py gpurun_out/ctr_r4b > gpurun_out/ctr_r4b/summary.txt 2>&1; cat gpurun_out/ctr_r4b/summary.txt
