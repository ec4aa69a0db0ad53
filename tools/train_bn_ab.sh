#!/bin/bash
# Training-step A/B of the fused train-mode BatchNorm (csrc/bn.hip, pnr.encoder.BatchNormTrain) against
# torch's nn.BatchNorm2d (MIOpen) + relu + add: alternating rounds on one box, scripts/bench_train.py
# 20 steps each.  Variants: 1 / 0 = PNR_FUSED_BN=1 / 0 eager; g1 / g0 = the same with the step
# replayed as one HIP graph (bench_train.py --graph: how much of the step is host launch cost).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for round in $(seq ${ROUNDS:-3}); do
  for v in ${VARIANTS:-"1 0"}; do
    flag=""; f=$v
    if [ "${v#g}" != "$v" ]; then flag="--graph"; f=${v#g}; fi
    echo -n "$round fused_bn=$v: "
    PNR_FUSED_BN=$f timeout -k 10 300 python scripts/bench_train.py --steps 20 --warmup 3 $flag 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" || exit $?
  done
done
