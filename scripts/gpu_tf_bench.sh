# TF-ME (ME_MCTF, TF level 2 of preset 8) at 4K: bench line + kernel trace
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/tf4k; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --workload 4k_tf_p8 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['value'], d['ms_per_step'], r['stages'], r['valu_sad'], d['cpu_baseline'], d['parity_vs_cpu'])" $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/kt" -o run --output-format csv -- python3 bench.py --workload 4k_tf_p8 --steps 20 --warmup 5 --no-cpu-baseline --band-steps 0 --no-upload --lanes 1 > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
head -8 $O/kt/run_kernel_stats.csv
