# SB-band part count sweep: parity at 2 and 3 parts, bench at 1..4
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SVTME_PARTS=3 timeout -k 10 600 python3 -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/parity_parts.log 2>&1 || { echo "parity failed"; tail -20 gpurun_out/parity_parts.log; exit 1; }
tail -2 gpurun_out/parity_parts.log
for p in 1 2 3 4; do
  SVTME_PARTS=$p timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_parts$p.json 2> gpurun_out/bench_parts$p.err || { echo "bench $p failed"; tail -5 gpurun_out/bench_parts$p.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_parts$p.json')); print('parts $p', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])"
done
