#!/bin/bash
# bench.py render legs (cfg3 headline + cfg2, and with COMPOSITE=1 the standalone composite leg) for
# libpnr.so variants in one box session, alternating.
#   VARIANTS="tagA default default:--unfused" [ROUNDS=2 STEPS=5 COMPOSITE=1] bash tools/bench_ab.sh
# (tag:args passes extra bench.py arguments to that variant; variants from scripts/build_variant.sh)
# (libpnr.so carries the soname libpnr.so, so libpnr_torch.so binds to the variant loaded first)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
comp="--no-composite"; [ -n "${COMPOSITE:-}" ] && comp=""
for round in $(seq ${ROUNDS:-2}); do
  for v in ${VARIANTS:-default}; do
    t=${v%%:*}; extra=""; [ "$t" != "$v" ] && extra=${v#*:}
    lib=pixel-nerf_amd/build/$t/libpnr.so
    [ "$t" = default ] && lib=pixel-nerf_amd/pnr/libpnr.so
    echo -n "$v: "
    PNR_LIB_PATH=$lib timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu --no-extra $comp \
        --no-compare --no-train $extra 2>/dev/null | python -c "
import json, sys
d = json.loads(sys.stdin.read()); c = d['cfg2']; k = d['kernel_ms']
s = 'cfg3 %.0f coarse %.3f fine %.3f frac %.4f | cfg2 %.0f fine %.3f frac %.4f | clk %.0f' % (
    d['value'], k['mlp_coarse'], k['mlp_fine'], d['roofline']['frac'], c['value'], c['kernel_ms']['mlp_fine'],
    c['roofline']['frac'], d.get('box_clock', {}).get('mhz_mean', 0))
if 'composite' in d:
    s += ' | composite %.4f ms frac %.4f, +weights %.4f ms frac %.4f' % (
        d['composite']['no_weights']['ms'], d['composite']['no_weights']['frac'],
        d['composite']['weights']['ms'], d['composite']['weights']['frac'])
print(s, flush=True)" || exit $?
  done
done
