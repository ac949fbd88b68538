# TF-ME records made by k_stage_c1 (no k_stage_e): the GPU suite, then the TF bench line
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/tf_direct; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 bench.py --workload 4k_tf_p8 --steps 50 --warmup 10 > $O/bench_tf.json 2> $O/bench_tf.err || { tail -20 $O/bench_tf.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('tf', d['value'], d['ms_per_step'], r['stages'], r['valu_sad']['frac'], d['parity_vs_cpu'])" $O/bench_tf.json
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('default', d['value'], d['with_sb_results'])" $O/bench_default.json
