cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_tests.sh > gpurun_out/r06c_tests.txt 2>&1 || { cat gpurun_out/r06c_tests.txt; exit 1; }
tail -3 gpurun_out/r06c_tests.txt
O=gpurun_out/r06c LIBS=prev bash scripts/gpu_ab_bench.sh
