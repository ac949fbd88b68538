# round-4 closing run of HEAD: smoke + the whole -m gpu suite, the default bench line, then the
# 4K p8 profile (kernel trace + PMC passes; the bench's `traffic` for this build's stage sources)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_close; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python3 scripts/first_job_probe.py > $O/first_job.json 2> $O/first_job.err || { tail $O/first_job.err; exit 1; }
cat $O/first_job.json
bash scripts/gpu_tests.sh > $O/gpu_tests_summary.txt 2>&1; rc=$?
cp gpurun_out/gpu_tests.log gpurun_out/smoke.log $O/ 2>/dev/null
tail -8 $O/gpu_tests_summary.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('default', d['value'], r['frac'], r['chip'], r['valu_sad']['frac'], d['upload']['pipelined_ms_per_picture'], d['band_8k']['step_ms'])" $O/bench_default.json
WL=4k_p8 TAG=r04_close/r04_4k_p8 bash scripts/gpu_profile.sh > $O/prof_4k_p8.log 2>&1 || { tail -20 $O/prof_4k_p8.log; exit 1; }
tail -1 $O/prof_4k_p8.log
timeout -k 10 600 python3 scripts/glue_rate.py $O/glue_rate.json 4k_p8_64f 4k_p8_16f 1080p_p8 > $O/glue_rate.log 2>&1 || { tail -20 $O/glue_rate.log; exit 1; }
cut -c1-200 $O/glue_rate.log
