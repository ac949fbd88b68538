cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06h
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06h/tests.log 2>&1 || { tail -30 gpurun_out/r06h/tests.log; exit 1; }
tail -3 gpurun_out/r06h/tests.log
LIBS=prev O=gpurun_out/r06h/ab bash scripts/gpu_ab_bench.sh || exit 1
O=gpurun_out/r06h/stamps SVTME_LIB=svt-av1-mirror_amd/libsvtme_stamp.so bash scripts/gpu_stamps.sh || exit 1
O=gpurun_out/r06h/glue bash scripts/gpu_glue.sh
