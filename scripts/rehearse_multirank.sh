#!/bin/bash
# Rehearse the N-rank bench code paths on a ONE-GPU box: 2 ranks on device 0 with the gloo
# backend (the driver's N-GPU runs use RCCL, one rank per GPU).  The cfg3 leg splits the
# 98,304-ray batch over the 2 ranks; the train leg all-reduces the gradients.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PNR_DIST_BACKEND=gloo PNR_FORCE_DEVICE=0
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 \
    > gpurun_out/rehearse_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep metric gpurun_out/rehearse_bench.log | cut -c1-600
exit $rc
