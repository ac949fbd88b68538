# smoke, then the full -m gpu suite (no -x: report every mismatch of one run).
# Exit status: the first failure of smoke (a mismatch is rc 1) or pytest.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
smoke_rc=$?
echo "smoke exit $smoke_rc"; tail -5 gpurun_out/smoke.log
# a fault, abort or time limit ends the call here; a bit-exact mismatch (rc 1) still runs the suite
if [ $smoke_rc -ne 0 ] && [ $smoke_rc -ne 1 ]; then exit $smoke_rc; fi
timeout -k 10 900 python3 -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread ${PYTEST_EXTRA:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "gpu tests exit $rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gpu_tests.log | tail -40
if [ $smoke_rc -ne 0 ]; then exit $smoke_rc; fi
exit $rc
