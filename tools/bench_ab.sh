#!/bin/bash
# bench.py render legs (cfg3 headline + cfg2) for libpnr.so variants in one box session,
# alternating.  Usage: VARIANTS="tagA default default:--unfused" bash tools/bench_ab.sh
# (tag:args passes extra bench.py arguments to that variant)
# (libpnr.so carries the soname libpnr.so, so libpnr_torch.so binds to the variant loaded first)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for round in $(seq ${ROUNDS:-2}); do
  for v in ${VARIANTS:-default}; do
    t=${v%%:*}; extra=""; [ "$t" != "$v" ] && extra=${v#*:}
    lib=pixel-nerf_amd/build/$t/libpnr.so
    [ "$t" = default ] && lib=pixel-nerf_amd/pnr/libpnr.so
    echo -n "$v: "
    PNR_LIB_PATH=$lib timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu --no-extra --no-composite \
        --no-compare --no-train $extra 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['cfg2']; print('cfg3', d['value'], d['kernel_ms']['mlp_coarse'], d['kernel_ms']['mlp_fine'], 'frac', d['roofline']['frac'], '| cfg2', c['value'], c['kernel_ms']['mlp_fine'], 'frac', c['roofline']['frac'])" || exit $?
  done
done
