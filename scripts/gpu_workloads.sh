# bench every BASELINE.json workload once (each with its CPU-baseline parity check)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for w in 1080p_p8 4k10_p6 8k_p8 4k_p8; do
  timeout -k 10 600 python3 bench.py --workload $w --steps 10 --warmup 3 > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { echo "bench $w failed $?"; tail -20 gpurun_out/bench_$w.err; exit 1; }
  echo "== $w"; cat gpurun_out/bench_$w.json
done
