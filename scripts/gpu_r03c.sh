# round-3 re-entry check of HEAD: smoke + the whole -m gpu suite (encoders included), the default
# bench line with its kernel trace, and the TF-ME bench line
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03c; mkdir -p $O
export TMPDIR=/tmp
bash scripts/gpu_tests.sh > $O/gpu_tests_summary.txt 2>&1; rc=$?
cp gpurun_out/gpu_tests.log gpurun_out/smoke.log $O/ 2>/dev/null
tail -8 $O/gpu_tests_summary.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('default', d['value'], d['roofline']['frac'], d['roofline']['valu_sad']['frac'])" $O/bench_default.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/kt_default" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --band-steps 0 --no-upload > $O/kt_default.log 2>&1 || { tail -20 $O/kt_default.log; exit 1; }
timeout -k 10 300 python3 bench.py --workload 4k_tf_p8 --steps 20 --warmup 5 > $O/bench_tf.json 2> $O/bench_tf.err || { tail -20 $O/bench_tf.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('tf', d['value'], d['ms_per_step'], r['stages'], r['valu_sad'], d['parity_vs_cpu'])" $O/bench_tf.json
