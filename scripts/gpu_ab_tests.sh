# GPU tests, then an A/B of the working tree's library against LIBS (scripts/gpu_ab_bench.sh).
# usage: [LIBS="prev"] [WL=4k_p8] [ROUNDS=2] [O=gpurun_out/abt] [TESTS="tests"] bash scripts/gpu_ab_tests.sh
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${O:-gpurun_out/abt}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
LIBS=${LIBS:-prev} O=$O/ab bash scripts/gpu_ab_bench.sh
