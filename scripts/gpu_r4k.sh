#!/bin/bash
# Round-4 session k: the render repeatability test under HBM contention; the eval encode forms
# (tools/encode_ab.py: module / folded graph / MIOpen fused graph); the training step with the
# encoder in channels-last (PNR_ENCODER_CL=1) against NCHW, alternating.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "== contention + encoder tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "contention or latent_channels_last or inference_trunk" \
    --timeout 120 --timeout-method thread > gpurun_out/tests_r4k.log 2>&1; rc=$?
tail -2 gpurun_out/tests_r4k.log; [ $rc = 0 ] || exit $rc
echo "== encode A/B"
timeout -k 10 300 python tools/encode_ab.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/encode_ab_r4k.txt; [ ${PIPESTATUS[0]} = 0 ] || exit 1
echo "== training A/B: encoder channels-last (1) vs NCHW (0)"
for round in 1 2; do
  for d in 0 1; do
    echo -n "encoder_cl=$d: "
    PNR_ENCODER_CL=$d timeout -k 10 300 python scripts/bench_train.py --steps 20 --warmup 3 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['loss'])" || exit 1
  done
done 2>&1 | tee gpurun_out/train_cl_r4k.txt
