# the closing build on the other BASELINE workloads: 4K 10-bit p6 and the 1080p 64x64 override
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_other; mkdir -p $O; export TMPDIR=/tmp
for WL in 4k10_p6 1080p_sa64; do
  timeout -k 10 300 python3 bench.py --workload $WL --steps 50 --warmup 10 > $O/bench_$WL.json 2> $O/bench_$WL.err || { tail -20 $O/bench_$WL.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], r['frac'], r['valu_sad'], {k: v['avg_ms'] for k, v in r['stages'].items()}, d['parity_vs_cpu'], d['cpu_baseline']['value'])" $O/bench_$WL.json
done
