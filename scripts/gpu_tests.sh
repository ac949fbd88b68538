# smoke, then the full -m gpu suite (no -x: report every mismatch of one run)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?
echo "smoke exit $rc"; tail -5 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python3 -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread ${PYTEST_EXTRA:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "gpu tests exit $rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gpu_tests.log | tail -40
exit $rc
