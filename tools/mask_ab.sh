#!/bin/bash
# A/B of the wave-major relu-mask save (csrc/mlp.hip save_mask / load_mask) against the [point][64 B]
# layout (the previous commit, scripts/build_variant.sh maskold HEAD~1): the training parity tests on
# the tree, tools/fwd_save_ab.py on both, and alternating cfg5 steps (scripts/bench_train.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
echo "== parity (tree)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 300 -p no:cacheprovider 2>&1 | tail -3
for lib in default maskold; do
  echo "== fwd_save_ab $lib"
  if [ $lib = default ]; then unset PNR_LIB_PATH; else export PNR_LIB_PATH=pixel-nerf_amd/build/$lib/libpnr.so; fi
  timeout -k 10 300 python tools/fwd_save_ab.py 2>/dev/null | grep round || exit 1
done
for round in 1 2 3; do
  for lib in default maskold; do
    echo -n "$round $lib: "
    if [ $lib = default ]; then unset PNR_LIB_PATH; else export PNR_LIB_PATH=pixel-nerf_amd/build/$lib/libpnr.so; fi
    timeout -k 10 300 python scripts/bench_train.py --steps 20 --warmup 3 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels']; print(d['value'], d['ms_per_step'], {n: v['ms_per_step'] for n, v in k.items()})" || exit 1
  done
done
