# the headline's dependence on the timed region: steps / warm-up sweep of the default workload
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04steps; mkdir -p $O; export TMPDIR=/tmp
for cfg in "50 10" "200 20" "200 200" "1000 20" "1000 200" "200 20"; do
  set -- $cfg
  timeout -k 10 200 python3 bench.py --steps $1 --warmup $2 --no-cpu-baseline --band-steps 0 --no-upload --no-sb-results --no-single-picture > $O/b_$1_$2.json 2> $O/b_$1_$2.err || { tail $O/b_$1_$2.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], round(d['value']/1e6,2), d['ms_per_step'], d['roofline']['frac'])" $O/b_$1_$2.json $1 $2
done
