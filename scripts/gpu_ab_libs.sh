# A/B of library builds: parity suite on each library, then the benches interleaved over rounds
# usage: LIBS="libsvtme_w0 libsvtme_w6" WLS="4k_p8 4k_p8_mixed" ROUNDS=3 bash scripts/gpu_ab_libs.sh
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab_libs; mkdir -p $O; export TMPDIR=/tmp
for L in $LIBS; do
  SVTME_LIB=svt-av1-mirror_amd/$L.so timeout -k 10 400 python3 -u -m pytest ${TESTS:-tests/test_configs.py tests/test_gpu_parity.py} -m gpu -x -q --timeout 200 --timeout-method thread > $O/t_$L.log 2>&1 || { tail -20 $O/t_$L.log; exit 1; }
  echo "$L $(tail -1 $O/t_$L.log)"
done
for r in $(seq 1 ${ROUNDS:-3}); do for WL in $WLS; do for L in $LIBS; do
  SVTME_LIB=svt-av1-mirror_amd/$L.so timeout -k 10 200 python3 bench.py --workload $WL --steps ${STEPS:-50} --warmup 10 --no-cpu-baseline --band-steps 0 > $O/b_${L}_${WL}_r$r.json 2> $O/b_${L}_${WL}_r$r.err || { tail $O/b_${L}_${WL}_r$r.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1].split('/')[-1], round(d['value']/1e6,2), {k: v['avg_ms'] for k, v in r['stages'].items()})" $O/b_${L}_${WL}_r$r.json
done; done; done
