# round-3 second batch: the real-time tune on both HME paths, k_fp_wide parity, low-delay encodes,
# then the k_fp_wide prologue A/B (wave 0 only vs every wave)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fpwide.py tests/test_encoder.py -k "golden or realtime or fp_wide or lowdelay" -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -12; [ $rc -eq 0 ] || exit $rc
LIBS="libsvtme libsvtme_w0off libsvtme_tq8w4" bash scripts/gpu_fpwide_ab.sh
