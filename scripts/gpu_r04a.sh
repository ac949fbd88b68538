# round 4, first GPU call: the upload-pipeline probe plain and under a kernel + memory-copy
# trace (timeline of copies vs searches), then smoke + the -m gpu suite on this round's box
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04a; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python3 scripts/upload_probe.py 40 > $O/probe.json 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
cat $O/probe.json
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$GRAFT_REPO_ROOT/$O/trace" -o run --output-format csv -- python3 scripts/upload_probe.py 20 > $O/probe_traced.log 2>&1 || { tail -20 $O/probe_traced.log; exit 1; }
tail -1 $O/probe_traced.log
bash scripts/gpu_tests.sh > $O/gpu_tests_summary.txt 2>&1; rc=$?
cp gpurun_out/gpu_tests.log gpurun_out/smoke.log $O/ 2>/dev/null
tail -4 $O/gpu_tests_summary.txt
exit $rc
