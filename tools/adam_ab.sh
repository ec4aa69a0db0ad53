#!/bin/bash
# pnr.optim.Adam (one pnr_adam_step launch) against torch's fused Adam on the cfg5 step: the parity
# test, then alternating scripts/bench_train.py runs with PNR_ADAM=pnr / torch.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -k adam -q --tb=short --timeout 200 -p no:cacheprovider 2>&1 | grep -E "^E |passed|failed|Error|test_gpu_train.py:[0-9]+" | head -30
for round in 1 2 3; do
  for v in pnr torch; do
    echo -n "$round adam=$v: "
    PNR_ADAM=$v timeout -k 10 300 python scripts/bench_train.py --steps 20 --warmup 3 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" || exit 1
  done
done
