cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/parity.log 2>&1; rc=$?; tail -2 gpurun_out/parity.log; [ $rc -eq 0 ] || exit $rc
for t in base default base default; do
  lib=pixel-nerf_amd/build/$t/libpnr.so; [ "$t" = default ] && lib=pixel-nerf_amd/pnr/libpnr.so
  echo -n "$t: "
  PNR_LIB_PATH=$lib timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --no-composite --no-compare 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extra_configs']; print(d['value'], e['cfg4_dtu_ns3_frame']['rays_per_s'], e['cfg3_nmr64_24frames']['rays_per_s'])" || exit $?
done
