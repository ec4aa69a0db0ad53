#!/bin/bash
# Round-4 session f: the eval encode as a BN-folded trunk replayed as one HIP graph
# (pnr.encoder.InferenceTrunk) -- its GPU tests, then rank 0's per-step work at N = 8 and N = 1
# (tools/shard_rehearsal.py) with the module's eager encode and with the graph, alternating.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
echo "== encoder tests"; date
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q \
    -k "latent_channels_last or inference_trunk or two_rank or gpus_2" \
    --timeout 300 --timeout-method thread > gpurun_out/enc_tests.log 2>&1; rc=$?
tail -3 gpurun_out/enc_tests.log; [ $rc = 0 ] || exit $rc
echo "== graph capture beside an RCCL process group"; date
timeout -k 10 120 python tools/graph_pg_check.py 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1
echo "== shard rehearsal"; date
: > gpurun_out/shards_r4f.jsonl
for round in 1 2; do
  for eager in 1 0; do
    ENCODER_EAGER=$eager timeout -k 10 300 python tools/shard_rehearsal.py 8 1 2>/dev/null >> gpurun_out/shards_r4f.jsonl || exit 1
  done
done
python - <<'EOF'
import json
for l in open("gpurun_out/shards_r4f.jsonl"):
    d = json.loads(l)
    print(d["world"], d["encoder"], "ms/step", d["ms_per_step"], "encode_ms", d["encode_ms"],
          "projected", d["projected_rays_per_s"], "mlp", d["render_kernel_ms_sum_per_chunk"])
EOF
