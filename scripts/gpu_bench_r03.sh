# default bench line (driver's command), the mixed-content line, and a kernel trace of each
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r03/bench_default.json 2> gpurun_out/r03/bench_default.err || { echo "bench failed $?"; tail -20 gpurun_out/r03/bench_default.err; exit 1; }
cat gpurun_out/r03/bench_default.json
timeout -k 10 600 python3 bench.py --workload 4k_p8_mixed --steps 50 --warmup 10 > gpurun_out/r03/bench_mixed.json 2> gpurun_out/r03/bench_mixed.err || { echo "bench mixed failed $?"; tail -20 gpurun_out/r03/bench_mixed.err; exit 1; }
cat gpurun_out/r03/bench_mixed.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r03/kt_mixed" -o run --output-format csv -- python3 bench.py --workload 4k_p8_mixed --steps 20 --warmup 5 --no-cpu-baseline --band-steps 0 --no-upload > gpurun_out/r03/kt_mixed.log 2>&1 || { echo "rocprof failed $?"; tail -20 gpurun_out/r03/kt_mixed.log; exit 1; }
find gpurun_out/r03 -name "*stats.csv"
