# the TF-ME batch test, then the mixed-content and 8K p8 profiles of the closing build
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_extra; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "mctf" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
WL=4k_p8_mixed TAG=r03_extra/r03e_4k_p8_mixed bash scripts/gpu_profile.sh > $O/prof_mixed.log 2>&1 || { tail -20 $O/prof_mixed.log; exit 1; }
tail -1 $O/prof_mixed.log
WL=8k_p8 TAG=r03_extra/r03e_8k_p8 bash scripts/gpu_profile.sh > $O/prof_8k.log 2>&1 || { tail -20 $O/prof_8k.log; exit 1; }
tail -1 $O/prof_8k.log
