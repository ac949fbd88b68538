# k_fp_wide A/B: parity of the wide configs for every library, then the 64x64-override bench, interleaved
# usage: LIBS="libsvtme libsvtme_w4" bash scripts/gpu_fpwide_ab.sh  (names under svt-av1-mirror_amd/)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fpwide_ab; mkdir -p $O
for L in $LIBS; do
  SVTME_LIB=svt-av1-mirror_amd/$L.so timeout -k 10 300 python3 -u -m pytest tests/test_configs.py tests/test_gpu_parity.py tests/test_gpu_fpwide.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/t_$L.log 2>&1 || { tail -20 $O/t_$L.log; exit 1; }
  echo "$L $(tail -1 $O/t_$L.log)"
done
for r in 1 2; do
  for L in $LIBS; do
    SVTME_LIB=svt-av1-mirror_amd/$L.so timeout -k 10 200 python3 -u bench.py --workload ${WL:-1080p_sa64} --steps 50 --warmup 10 --no-cpu-baseline > $O/b_${L}_r$r.json 2> $O/b_${L}_r$r.err || { tail $O/b_${L}_r$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], {k: v['avg_ms'] for k, v in r['stages'].items()}, r['valu_sad']['frac'])" $O/b_${L}_r$r.json
  done
done
