#!/bin/bash
# Round-4 session g: the eval encode forms (tools/encode_ab.py: module / folded graph / MIOpen
# fused conv+relu graph), the encoder GPU tests, and the N = 8 shard rehearsal with the default.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "== encode A/B"; date
timeout -k 10 300 python tools/encode_ab.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/encode_ab.txt; [ ${PIPESTATUS[0]} = 0 ] || exit 1
echo "== encoder tests"; date
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "latent_channels_last or inference_trunk" \
    --timeout 120 --timeout-method thread > gpurun_out/enc_tests_g.log 2>&1; rc=$?
tail -2 gpurun_out/enc_tests_g.log; [ $rc = 0 ] || exit $rc
echo "== shard rehearsal"; date
: > gpurun_out/shards_r4g.jsonl
for round in 1 2; do
  for eager in 1 0; do
    ENCODER_EAGER=$eager timeout -k 10 300 python tools/shard_rehearsal.py 8 2>/dev/null >> gpurun_out/shards_r4g.jsonl || exit 1
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/shards_r4g.jsonl"):
    d = json.loads(l)
    print(d["world"], d["encoder"], "ms/step", d["ms_per_step"], "encode_ms", d["encode_ms"],
          "projected", d["projected_rays_per_s"], "mlp", d["render_kernel_ms_sum_per_chunk"])
PY
