#!/bin/bash
# Round-4 session j: weight gradients on a side stream (pnr.train.DEFER_WGRAD) -- training GPU
# tests, then the training bench alternating PNR_DEFER_WGRAD=0 / 1.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "== training GPU tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/train_tests_r4j.log 2>&1; rc=$?; tail -2 gpurun_out/train_tests_r4j.log; [ $rc = 0 ] || exit $rc
echo "== training A/B: weight gradients deferred to a side stream (1) vs in order (0)"
for round in 1 2 3; do
  for d in 0 1; do
    echo -n "defer=$d: "
    PNR_DEFER_WGRAD=$d timeout -k 10 300 python scripts/bench_train.py --steps 20 --warmup 3 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], {k: v['ms_per_step'] for k, v in d['roofline']['kernels'].items()})" || exit 1
  done
done 2>&1 | tee gpurun_out/train_ab_r4j.txt
