# bench every workload at the driver's window (--steps 20 --warmup 5 in a fresh process; CPU leg and
# parity check included): the DESIGN.md 4 table (profiles/r05_workloads/)
# usage: [WLS="..."] [O=gpurun_out/workloads] bash scripts/gpu_workloads.sh
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${O:-gpurun_out/workloads}; mkdir -p $O
for w in ${WLS:-4k_p8 4k_p8_mixed 8k_p8 1080p_sa64 4k10_p6 4k_tf_p8}; do
  timeout -k 10 300 python3 -u bench.py --workload $w > $O/$w.json 2> $O/$w.err || { echo "bench $w failed"; tail -20 $O/$w.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], r['frac'], r['valu_sad']['frac'], {k: v['avg_ms'] for k, v in r['stages'].items()}, (d.get('steady_state') or {}).get('value'), d['cpu_baseline']['value'], d['parity_vs_cpu'])" $O/$w.json $w
done
