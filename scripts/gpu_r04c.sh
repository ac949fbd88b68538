# round 4: the glue-served ME rate with primed kernels and linear uploads (per-job trace), the default bench line
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 scripts/glue_rate.py $O/glue_rate.json > $O/glue_rate.log 2>&1 || { tail -20 $O/glue_rate.log; exit 1; }
cat $O/glue_rate.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('default', d['value'], d['roofline']['frac'], d['roofline']['bound'], d['roofline']['chip'], d['upload'], d['band_8k'])" $O/bench_default.json
