#!/bin/bash
# Round-4 session l: channels-last encoder trunk (NHWC latent kernel, unfused folded eval trunk):
# every GPU test + smoke + bench, then rank 0's N = 8 share (tools/shard_rehearsal.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
BENCH_STEPS=10 bash scripts/gpu_check.sh || exit $?
echo "== shard rehearsal"
: > gpurun_out/shards_r4l.jsonl
for round in 1 2; do
  for w in 8 1; do
    timeout -k 10 300 python tools/shard_rehearsal.py $w 2>/dev/null >> gpurun_out/shards_r4l.jsonl || exit 1
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/shards_r4l.jsonl"):
    d = json.loads(l)
    print(d["world"], d["encoder"], "ms/step", d["ms_per_step"], "encode_ms", d["encode_ms"],
          "projected", d["projected_rays_per_s"], "mlp", d["render_kernel_ms_sum_per_chunk"])
PY
