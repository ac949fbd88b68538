# k_fp_wide bring-up: parity tests of the wide full-pel paths, then the 64x64-override
# bench with and without it (SVTME_NO_FP_WIDE=1: k_stage_c1)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fpwide
timeout -k 10 600 python3 -u -m pytest tests/test_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fpwide/tests.log 2>&1
rc=$?; tail -5 gpurun_out/fpwide/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 0 1; do
    if [ $v = 1 ]; then export SVTME_NO_FP_WIDE=1; else unset SVTME_NO_FP_WIDE; fi
    timeout -k 10 200 python3 -u bench.py --workload 1080p_sa64 --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/fpwide/bench_v${v}_r$r.json 2> gpurun_out/fpwide/bench_v${v}_r$r.err || { tail gpurun_out/fpwide/bench_v${v}_r$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], r['stages'], r['valu_sad'])" gpurun_out/fpwide/bench_v${v}_r$r.json
  done
done
