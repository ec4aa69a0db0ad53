#!/bin/bash
# Round-4 session a: GPU tests + smoke (scripts/gpu_check.sh, no bench), then the same-box A/B of the
# pruned mlp.hip against the pre-prune kernel source (build/pre: 535a5a3's mlp.hip with this tree's
# other sources), render legs and the training step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
NO_BENCH=1 bash scripts/gpu_check.sh || exit $?
echo "== render A/B"; date
VARIANTS="pre default" ROUNDS=2 STEPS=5 bash tools/bench_ab.sh > gpurun_out/ab_prune.txt 2>&1; rc=$?
cat gpurun_out/ab_prune.txt; [ $rc -eq 0 ] || exit $rc
echo "== train A/B"; date
VARIANTS="pre default" STEPS=20 bash tools/train_lib_ab.sh > gpurun_out/ab_prune_train.txt 2>&1; rc=$?
cat gpurun_out/ab_prune_train.txt; exit $rc
