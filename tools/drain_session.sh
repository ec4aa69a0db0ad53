#!/bin/bash
# A/B of the LDS-drained activation save (PNR_SAVE_DRAIN, csrc/mlp.hip Drain) against the publish-burst
# save: the variant library pixel-nerf_amd/build/drain/libpnr.so (scripts/build_variant.sh drain WORKTREE
# -DPNR_SAVE_DRAIN=1).  1) the training parity tests on the variant; 2) tools/fwd_save_ab.py on both;
# 3) alternating cfg5 training steps (scripts/bench_train.py, 20 steps) on both.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
V=pixel-nerf_amd/build/drain/libpnr.so
echo "== parity (drain)"
PNR_LIB_PATH=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 300 -p no:cacheprovider 2>&1 | tail -3 || exit 1
for lib in default drain; do
  echo "== fwd_save_ab $lib"
  if [ $lib = drain ]; then export PNR_LIB_PATH=$V; else unset PNR_LIB_PATH; fi
  timeout -k 10 300 python tools/fwd_save_ab.py 2>/dev/null | grep round || exit 1
done
unset PNR_LIB_PATH
for round in 1 2 3; do
  for lib in default drain; do
    echo -n "$round $lib: "
    if [ $lib = drain ]; then export PNR_LIB_PATH=$V; else unset PNR_LIB_PATH; fi
    timeout -k 10 300 python scripts/bench_train.py --steps 20 --warmup 3 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels']; print(d['value'], d['ms_per_step'], {n: v['ms_per_step'] for n, v in k.items()})" || exit 1
  done
done
