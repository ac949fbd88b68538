# k_fp_wide A/B in steady state, round 7: no SAD barrier on whole sets (the scheduler interleaves sets; product) against HEAD
# (barrier after every set)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04fpab7; mkdir -p $O; export TMPDIR=/tmp
for L in libsvtme libsvtme_head; do
  SVTME_LIB=svt-av1-mirror_amd/$L.so timeout -k 10 400 python3 -u -m pytest tests/test_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/t_$L.log 2>&1 || { tail -20 $O/t_$L.log; exit 1; }
  echo "$L $(tail -1 $O/t_$L.log)"
done
for r in 1 2 3; do for L in libsvtme libsvtme_head; do
  SVTME_LIB=svt-av1-mirror_amd/$L.so timeout -k 10 200 python3 bench.py --workload 1080p_sa64 --no-cpu-baseline --band-steps 0 --no-upload --no-sb-results --no-single-picture > $O/b_${L}_r$r.json 2> $O/b_${L}_r$r.err || { tail $O/b_${L}_r$r.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1].split('/')[-1], round(d['value']/1e6,3), r['valu_sad']['frac'], {k: v['avg_ms'] for k, v in r['stages'].items()})" $O/b_${L}_r$r.json
done; done
