cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu --no-extra --no-composite > gpurun_out/bench_proj.log 2>&1 || exit $?
tail -1 gpurun_out/bench_proj.log
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu --no-extra --no-composite --no-latent-proj --no-compare > gpurun_out/bench_noproj.log 2>&1 || exit $?
tail -1 gpurun_out/bench_noproj.log
