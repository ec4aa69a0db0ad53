#!/bin/bash
# Round-4 session e: the relu folded into the publish split (build/rtz, -DPNR_RTZ_RELU: hi part by
# round-toward-zero + packed fp16 relu, lo part by the residual's clamp) -- parity tests and the
# precision study on it, render and training A/B against HEAD; then a training-step profile with
# the region timeline (tools/train_step_breakdown.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
RTZ=pixel-nerf_amd/build/rtz/libpnr.so
echo "== rtz parity"; date
PNR_LIB_PATH=$RTZ timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/rtz_parity.log 2>&1; rc=$?
tail -3 gpurun_out/rtz_parity.log; [ $rc = 0 ] || exit $rc
echo "== precision"; date
for v in default rtz; do
  lib=pixel-nerf_amd/pnr/libpnr.so; [ $v = rtz ] && lib=$RTZ
  PNR_LIB_PATH=$lib timeout -k 10 300 python tools/precision_study.py > gpurun_out/prec_$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/prec_$v.json')); print('$v', d['f16x3'], d['fp32'])"
done
echo "== render A/B"; date
VARIANTS="rtz default" ROUNDS=2 bash tools/bench_ab.sh || exit 1
echo "== train A/B"; date
for round in 1 2; do
  for v in rtz default; do
    lib=pixel-nerf_amd/pnr/libpnr.so; [ $v = rtz ] && lib=$RTZ
    echo -n "$v: "
    PNR_LIB_PATH=$lib timeout -k 10 300 python scripts/bench_train.py --steps 10 --warmup 3 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" || exit 1
  done
done
echo "== train profile"; date
bash tools/profile_train.sh r4e
