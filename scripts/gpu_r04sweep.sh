# every BASELINE workload with the default steps / warm-up (steady state), CPU baseline + parity each
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04sweep; mkdir -p $O; export TMPDIR=/tmp
for WL in 4k_p8_mixed 8k_p8 1080p_sa64 4k10_p6 4k_tf_p8; do
  timeout -k 10 300 python3 bench.py --workload $WL --band-steps 0 > $O/bench_$WL.json 2> $O/bench_$WL.err || { tail -20 $O/bench_$WL.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1].split('/')[-1], round(d['value']/1e6,2), r['frac'], r['chip']['frac'], r['valu_sad']['frac'], {k: v['avg_ms'] for k, v in r['stages'].items()}, d['parity_vs_cpu'], d['cpu_baseline']['value'])" $O/bench_$WL.json
done
