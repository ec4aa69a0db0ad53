#!/bin/bash
# A/B of write-through (sc1) activation-save stores (PNR_SAVE_WT, csrc/mlp.hip save_store16) against
# plain stores: the variant library pixel-nerf_amd/build/savewt/libpnr.so (scripts/build_variant.sh
# savewt WORKTREE -DPNR_SAVE_WT=1).  1) the training parity tests on the variant; 2) tools/fwd_save_ab.py
# on both; 3) alternating cfg5 training steps (scripts/bench_train.py, 20 steps) on both.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
V=pixel-nerf_amd/build/savewt/libpnr.so
echo "== parity (savewt)"
PNR_LIB_PATH=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 300 -p no:cacheprovider 2>&1 | tail -3
for lib in default savewt; do
  echo "== fwd_save_ab $lib"
  if [ $lib = savewt ]; then export PNR_LIB_PATH=$V; else unset PNR_LIB_PATH; fi
  timeout -k 10 300 python tools/fwd_save_ab.py 2>/dev/null | grep round || exit 1
done
unset PNR_LIB_PATH
for round in 1 2 3; do
  for lib in default savewt; do
    echo -n "$round $lib: "
    if [ $lib = savewt ]; then export PNR_LIB_PATH=$V; else unset PNR_LIB_PATH; fi
    timeout -k 10 300 python scripts/bench_train.py --steps 20 --warmup 3 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels']; print(d['value'], d['ms_per_step'], {n: v['ms_per_step'] for n, v in k.items()})" || exit 1
  done
done
