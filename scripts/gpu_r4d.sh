#!/bin/bash
# Round-4 session d: the training step's non-MLP time -- the encoder trunk in
# NCHW / channels_last / native-conv forms (tools/encoder_probe.py), and the whole step eager
# against one HIP graph per step, alternating on one box.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "== encoder probe"; date
timeout -k 10 300 python tools/encoder_probe.py > gpurun_out/encoder_probe.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/encoder_probe.txt; [ $rc = 0 ] || exit $rc
echo "== train eager / graph"; date
for round in 1 2; do
  for v in eager graph; do
    flag=""; [ $v = graph ] && flag=--graph
    echo -n "$v: "
    timeout -k 10 300 python scripts/bench_train.py --steps 10 --warmup 3 $flag 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" || exit 1
  done
done
