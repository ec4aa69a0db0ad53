#!/bin/bash
# Training-step A/B of libpnr.so variants in one box session, alternating:
#   VARIANTS="tagA default" bash tools/train_lib_ab.sh
# (tag = pixel-nerf_amd/build/<tag>/libpnr.so from scripts/build_variant.sh; default = in-tree)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for round in 1 2 3; do
  for t in ${VARIANTS:-default}; do
    lib=pixel-nerf_amd/build/$t/libpnr.so
    [ "$t" = default ] && lib=pixel-nerf_amd/pnr/libpnr.so
    echo -n "$t: "
    PNR_LIB_PATH=$lib timeout -k 10 300 python scripts/bench_train.py --steps ${STEPS:-20} --warmup 3 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" || exit $?
  done
done
