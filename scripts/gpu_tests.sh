# the full -m gpu suite, as the driver runs it
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -m pytest tests -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests exit $rc"; tail -25 gpurun_out/gpu_tests.log
exit $rc
