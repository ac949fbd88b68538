# 8x8 full-pel area fast path (fp_rows32_8x8) A/B: MCTF / golden parity with the product library,
# then the TF-ME and 10-bit benches with it and without it (libsvtme_nofp8: -DSVTME_FP8X8=0)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fp8x8; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_encoder.py -k "mctf or tf or golden or 360p_p8 or ra360 or 240p" -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -12; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for L in libsvtme libsvtme_nofp8; do for WL in 4k_tf_p8 4k10_p6; do
  SVTME_LIB=svt-av1-mirror_amd/$L.so timeout -k 10 200 python3 bench.py --workload $WL --steps 20 --warmup 5 --no-cpu-baseline --band-steps 0 > $O/b_${L}_${WL}_r$r.json 2> $O/b_${L}_${WL}_r$r.err || { tail $O/b_${L}_${WL}_r$r.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], {k: v['avg_ms'] for k, v in r['stages'].items()})" $O/b_${L}_${WL}_r$r.json
done; done; done
