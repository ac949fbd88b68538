# k_fp_wide set width A/B: FPW_TQ 4 / 6 / 8 builds, parity of the 64x64-override config, bench
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fpwide_tq
for L in libsvtme_tq4 libsvtme libsvtme_tq8; do
  SVTME_LIB=svt-av1-mirror_amd/$L.so timeout -k 10 300 python3 -u -m pytest tests/test_configs.py -m gpu -x -q -k "sa64" --timeout 200 --timeout-method thread > gpurun_out/fpwide_tq/t_$L.log 2>&1 || { tail -20 gpurun_out/fpwide_tq/t_$L.log; exit 1; }
  tail -1 gpurun_out/fpwide_tq/t_$L.log
done
for r in 1 2; do
  for L in libsvtme_tq4 libsvtme libsvtme_tq8; do
    SVTME_LIB=svt-av1-mirror_amd/$L.so timeout -k 10 200 python3 -u bench.py --workload 1080p_sa64 --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/fpwide_tq/b_${L}_r$r.json 2> gpurun_out/fpwide_tq/b_${L}_r$r.err || { tail gpurun_out/fpwide_tq/b_${L}_r$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], r['stages'], r['valu_sad']['frac'])" gpurun_out/fpwide_tq/b_${L}_r$r.json
  done
done
