#!/bin/bash
# Round-4 session i: publish-split register plan A/B -- the next GEMM's weight ring primed after
# the split (PNR_LATE_PRIME), the split's row groups computed side by side (PNR_SPLIT_ILP), both;
# bitwise check of each against the default, then bench_ab alternating.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for t in default late_prime split_ilp ilp_late; do
  lib=pixel-nerf_amd/build/$t/libpnr.so; [ $t = default ] && lib=pixel-nerf_amd/pnr/libpnr.so
  PNR_LIB_PATH=$lib timeout -k 10 180 python tools/bitwise_ab.py save gpurun_out/bw_$t.pt 2>&1 | grep -v amdgpu.ids | tail -1
  [ ${PIPESTATUS[0]} = 0 ] || exit 1
done
for t in late_prime split_ilp ilp_late; do
  echo -n "$t vs default: "; python tools/bitwise_ab.py cmp gpurun_out/bw_default.pt gpurun_out/bw_$t.pt | tail -1
done
rm -f gpurun_out/bw_*.pt
VARIANTS="default late_prime split_ilp ilp_late" ROUNDS=2 bash tools/bench_ab.sh 2>&1 | tee gpurun_out/ab_r4i.txt
echo "== deferred weight-gradient test + training gradient tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/train_tests_r4i.log 2>&1; rc=$?; tail -2 gpurun_out/train_tests_r4i.log; [ $rc = 0 ] || exit $rc
echo "== training A/B: weight gradients deferred to a side stream (1) vs in order (0)"
for round in 1 2; do
  for d in 0 1; do
    echo -n "defer=$d: "
    PNR_DEFER_WGRAD=$d timeout -k 10 300 python scripts/bench_train.py --steps 10 --warmup 3 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'])" || exit 1
  done
done 2>&1 | tee gpurun_out/train_ab_r4i.txt
