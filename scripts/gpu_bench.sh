# bench + rocprofv3 kernel trace (+ PMC passes); stops at the first failing GPU step
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed $?"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_kt" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_kt.log 2>&1 || { echo "rocprof kt failed $?"; tail -20 gpurun_out/prof_kt.log; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$GRAFT_REPO_ROOT/gpurun_out/prof_fetch" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --kernel-samples 2 > gpurun_out/prof_fetch.log 2>&1 || { echo "rocprof fetch failed $?"; tail -20 gpurun_out/prof_fetch.log; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$GRAFT_REPO_ROOT/gpurun_out/prof_write" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --kernel-samples 2 > gpurun_out/prof_write.log 2>&1 || { echo "rocprof write failed $?"; tail -20 gpurun_out/prof_write.log; exit 1; }
find gpurun_out -name "*.csv" | head -20
