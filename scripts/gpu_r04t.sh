# round 4: 4 MB warm-up copies at context creation -- first-job latency (+ HIP API trace), glue rate
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04t; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 120 python3 scripts/first_job_probe.py > $O/first_job.json 2> $O/first_job.err || { tail $O/first_job.err; exit 1; }
cat $O/first_job.json
timeout -k 10 180 rocprofv3 --hip-trace --memory-copy-trace --stats -d "$GRAFT_REPO_ROOT/$O/trace" -o run --output-format csv -- python3 scripts/first_job_probe.py > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
timeout -k 10 300 python3 -u -m pytest tests/test_encoder.py tests/test_pack.py -m gpu -q --timeout 150 --timeout-method thread > $O/enc.log 2>&1 || { tail -30 $O/enc.log; exit 1; }
tail -1 $O/enc.log
timeout -k 10 600 python3 scripts/glue_rate.py $O/glue_rate.json 4k_p8_64f 4k_p8_16f 1080p_p8 > $O/glue_rate.log 2>&1 || { tail -20 $O/glue_rate.log; exit 1; }
cut -c1-200 $O/glue_rate.log
