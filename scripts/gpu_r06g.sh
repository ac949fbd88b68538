cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_tests.sh > gpurun_out/r06g_tests.txt 2>&1 || { tail -40 gpurun_out/r06g_tests.txt; exit 1; }
tail -3 gpurun_out/r06g_tests.txt
O=gpurun_out/r06g LIBS=prev bash scripts/gpu_ab_bench.sh || exit 1
O=gpurun_out/r06g_stamps bash scripts/gpu_stamps.sh
