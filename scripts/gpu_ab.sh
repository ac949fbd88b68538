export TMPDIR=/tmp; O=gpurun_out/r05m; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_rtcd.py > $O/t.log 2>&1; rc=$?; tail -3 $O/t.log; exit $rc
