# round 4: first-job latency (an empty kernel launched per code object at context creation)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04q; mkdir -p $O; export TMPDIR=/tmp
for k in 1 2; do timeout -k 10 120 python3 scripts/first_job_probe.py > $O/first_job_$k.json 2> $O/first_job_$k.err || { tail $O/first_job_$k.err; exit 1; }; cat $O/first_job_$k.json; done
timeout -k 10 300 python3 -u -m pytest tests/test_encoder.py tests/test_pack.py -m gpu -q --timeout 150 --timeout-method thread > $O/enc.log 2>&1 || { tail -30 $O/enc.log; exit 1; }
tail -1 $O/enc.log
timeout -k 10 600 python3 scripts/glue_rate.py $O/glue_rate.json 4k_p8_64f 4k_p8_16f 1080p_p8 > $O/glue_rate.log 2>&1 || { tail -20 $O/glue_rate.log; exit 1; }
cut -c1-200 $O/glue_rate.log
