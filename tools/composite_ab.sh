#!/bin/bash
# Standalone composite kernel (bench.py composite_roofline: 1 M rays x 128 samples) for libpnr.so
# variants, alternating: VARIANTS="default comp2" bash tools/composite_ab.sh.  The round-5 variants
# (the chunked layout) builds from tools/patches/composite_variants.diff, e.g.
#   PATCH=tools/patches/composite_variants.diff scripts/build_variant.sh compc WORKTREE
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for round in $(seq ${ROUNDS:-3}); do
  for t in ${VARIANTS:-default comp2}; do
    lib=pixel-nerf_amd/build/$t/libpnr.so
    [ "$t" = default ] && lib=pixel-nerf_amd/pnr/libpnr.so
    echo -n "$round $t: "
    PNR_LIB_PATH=$lib timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu --no-extra --no-train \
        --no-cfg2 --no-clock 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read())['composite']; print({k: (v['ms'], v['achieved'], v['frac']) for k, v in d.items()})" || exit $?
  done
done
