# round 4, k_fp_wide with whole sets in a straight loop, folded every two sets: the whole GPU suite, the default line,
# the 4K p8 profile for this build's code_sha, then 3 runs of the 1080p override
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04final3; mkdir -p $O; export TMPDIR=/tmp
bash scripts/gpu_tests.sh > $O/gpu_tests_summary.txt 2>&1; rc=$?
cp gpurun_out/gpu_tests.log gpurun_out/smoke.log $O/ 2>/dev/null
tail -4 $O/gpu_tests_summary.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('default', d['value'], r['frac'], r['chip']['frac'], r['valu_sad']['frac'], d['upload']['pipelined_ms_per_picture'], d['band_8k']['step_ms'])" $O/bench_default.json
WL=4k_p8 TAG=r04final3/r04_4k_p8 bash scripts/gpu_profile.sh > $O/prof_4k_p8.log 2>&1 || { tail -20 $O/prof_4k_p8.log; exit 1; }
tail -1 $O/prof_4k_p8.log
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --workload 1080p_sa64 --no-cpu-baseline --band-steps 0 --no-upload --no-sb-results --no-single-picture > $O/b_sa64_r$r.json 2> $O/b_sa64_r$r.err || { tail $O/b_sa64_r$r.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1].split('/')[-1], round(d['value']/1e6,3), r['valu_sad']['frac'], {k: v['avg_ms'] for k, v in r['stages'].items()})" $O/b_sa64_r$r.json
done
