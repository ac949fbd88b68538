# round-3 closing run of HEAD: smoke + the whole -m gpu suite, the default bench line with its
# kernel trace, then bench + kernel trace + PMC passes (HBM traffic) of 4K p8 and of the TF-ME workload
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_close2; mkdir -p $O
export TMPDIR=/tmp
bash scripts/gpu_tests.sh > $O/gpu_tests_summary.txt 2>&1; rc=$?
cp gpurun_out/gpu_tests.log gpurun_out/smoke.log $O/ 2>/dev/null
tail -8 $O/gpu_tests_summary.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('default', d['value'], d['roofline']['frac'], d['roofline']['valu_sad']['frac'])" $O/bench_default.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/kt_default" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --band-steps 0 --no-upload > $O/kt_default.log 2>&1 || { tail -20 $O/kt_default.log; exit 1; }
WL=4k_p8 TAG=r03_close2/r03f_4k_p8 bash scripts/gpu_profile.sh > $O/prof_4k_p8.log 2>&1 || { tail -20 $O/prof_4k_p8.log; exit 1; }
tail -2 $O/prof_4k_p8.log
WL=4k_tf_p8 TAG=r03_close2/r03f_4k_tf_p8 bash scripts/gpu_profile.sh > $O/prof_4k_tf_p8.log 2>&1 || { tail -20 $O/prof_4k_tf_p8.log; exit 1; }
tail -2 $O/prof_4k_tf_p8.log
