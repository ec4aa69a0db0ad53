#!/bin/bash
# Training-step A/B (one box, alternating rounds, scripts/bench_train.py 20 steps); the variants need
# tools/patches/defer_wgrad_cumask.diff / save_nt.diff applied (rejected in round 5, profiles/r5b):
#   base    the weight gradients in order on the launch stream
#   defer   k_wgrad_h on a side stream beside the encoder backward (pnr.train DEFER_WGRAD)
#   m<N>    defer, the side stream on the first N CUs (PNR_WGRAD_CUMASK=N, hipExtStreamCreateWithCUMask)
#   x<S>    defer, the side stream on every CU but each S-th mask bit
#   nt      libpnr built with -DPNR_SAVE_NT=1 (streaming stores of the activation save / dY slots):
#           pixel-nerf_amd/build/savent/libpnr.so (scripts/build_variant.sh savent WORKTREE -DPNR_SAVE_NT=1)
#   nt+<v>  nt combined with variant v
cd "${GRAFT_REPO_ROOT:-/root/repo}"
VARIANTS=${VARIANTS:-"base defer m224 x8 nt"}
for round in $(seq ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    env="PNR_DEFER_WGRAD=0"
    w=$v
    if [ "${v#nt+}" != "$v" ] || [ "$v" = nt ]; then
      env="$env PNR_LIB_PATH=pixel-nerf_amd/build/savent/libpnr.so"; w=${v#nt}; w=${w#+}
    fi
    case $w in
      ""|base) ;;
      defer) env="$env PNR_DEFER_WGRAD=1";;
      m*) env="$env PNR_DEFER_WGRAD=1 PNR_WGRAD_CUMASK=${w#m}";;
      x*) env="$env PNR_DEFER_WGRAD=1 PNR_WGRAD_CUMASK=$w";;
    esac
    echo -n "$round $v: "
    env $env timeout -k 10 300 python scripts/bench_train.py --steps 20 --warmup 3 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels']; print(d['value'], d['ms_per_step'], {n: v['ms_per_step'] for n, v in k.items()})" || exit $?
  done
done
