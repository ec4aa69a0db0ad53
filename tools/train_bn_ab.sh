#!/bin/bash
# Training-step A/B of the fused train-mode BatchNorm (csrc/bn.hip, pnr.encoder.BatchNormTrain) against
# torch's nn.BatchNorm2d (MIOpen) + relu + add: alternating rounds on one box, scripts/bench_train.py
# 20 steps each; PNR_FUSED_BN=1 / 0.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for round in $(seq ${ROUNDS:-3}); do
  for v in ${VARIANTS:-"1 0"}; do
    echo -n "$round fused_bn=$v: "
    PNR_FUSED_BN=$v timeout -k 10 300 python scripts/bench_train.py --steps 20 --warmup 3 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" || exit $?
  done
done
