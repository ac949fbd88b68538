# iteration loop: parity tests, bench, (optional) stamped run and SQ counters
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/parity.log 2>&1
rc=$?; echo "parity exit $rc"; tail -15 gpurun_out/parity.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
if [ -n "$STAMPS" ]; then
SVTME_LIB=libsvtme_stamps.so timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --kernel-samples 1 --no-cpu-baseline > gpurun_out/stamps.json 2> gpurun_out/stamps.err || { echo "stamps failed"; tail -20 gpurun_out/stamps.err; exit 1; }
grep stamps gpurun_out/stamps.err
fi
if [ -n "$KT" ]; then
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_kt" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_kt.log 2>&1 || { echo "rocprof kt failed $?"; tail -20 gpurun_out/prof_kt.log; exit 1; }
cat gpurun_out/prof_kt/run_kernel_stats.csv
fi
if [ -n "$SQ" ]; then bash scripts/gpu_sq.sh; fi
