# bench sweep of submission shapes: pictures per step x pictures per launch x lanes
# usage: WL=4k_p8 SHAPES="4:16:1 4:2:2 4:1:2" [STEPS=100 WARMUP=20 BENCH_ARGS=...] bash scripts/gpu_lanes.sh   (P:LP:lanes)
cd "$GRAFT_REPO_ROOT"
WL=${WL:-4k_p8}
O=gpurun_out/lanes_$WL
mkdir -p $O
for sh in ${SHAPES:-4:16:1 4:4:2 4:2:2 4:1:2 8:4:2 8:2:2}; do
  IFS=: read P LP L <<< "$sh"
  timeout -k 10 180 python3 -u bench.py --workload $WL --pictures $P --launch-pictures $LP --lanes $L \
    --steps ${STEPS:-100} --warmup ${WARMUP:-20} --no-cpu-baseline --no-upload --no-single-picture ${BENCH_ARGS:-} \
    > $O/p${P}_lp${LP}_l${L}.json 2> $O/p${P}_lp${LP}_l${L}.err || { echo "bench $sh failed"; tail -20 $O/p${P}_lp${LP}_l${L}.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['frac'])" \
    $O/p${P}_lp${LP}_l${L}.json "$sh"
done
