# round 4: every kernel primed on an empty batch at context creation -- first-job latency, the whole
# GPU suite, glue rate
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04r; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 120 python3 scripts/first_job_probe.py > $O/first_job.json 2> $O/first_job.err || { tail $O/first_job.err; exit 1; }
cat $O/first_job.json
bash scripts/gpu_tests.sh > $O/gpu_tests_summary.txt 2>&1; rc=$?
cp gpurun_out/gpu_tests.log gpurun_out/smoke.log $O/ 2>/dev/null
tail -4 $O/gpu_tests_summary.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 scripts/glue_rate.py $O/glue_rate.json 4k_p8_64f 4k_p8_16f 1080p_p8 > $O/glue_rate.log 2>&1 || { tail -20 $O/glue_rate.log; exit 1; }
cut -c1-200 $O/glue_rate.log
