export TMPDIR=/tmp; O=gpurun_out/r05cc; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "zero_copy or upload or pyramid" > $O/t.log 2>&1; rc=$?; tail -3 $O/t.log; exit $rc
