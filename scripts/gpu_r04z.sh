# round 4, last check of HEAD: smoke + the default bench line (as the driver runs them)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04z; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('default', d['value'], r['frac'], r['chip']['frac'], r['traffic'], r.get('traffic_source'), r['valu_sad']['frac'], d['upload']['pipelined_ms_per_picture'], d['band_8k']['step_ms'], d['cpu_baseline']['value'])" $O/bench_default.json
