cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_tests.sh > gpurun_out/r06f_tests.txt 2>&1 || { tail -40 gpurun_out/r06f_tests.txt; exit 1; }
tail -3 gpurun_out/r06f_tests.txt
O=gpurun_out/r06f LIBS=prev bash scripts/gpu_ab_bench.sh || exit 1
O=gpurun_out/r06f_p6 WL=4k10_p6 LIBS=noL2 bash scripts/gpu_ab_bench.sh || exit 1
O=gpurun_out/r06f_stamps WLS="4k_p8 4k10_p6" bash scripts/gpu_stamps.sh
