# round 4: the whole -m gpu suite on HEAD's library, the A/B of the A1 / L1 tile -> search maps
# (libsvtme_base.so: the binary-search build) on 4K p8 and the mixed content, the glue rate of a 64-frame 4K encode
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04f; mkdir -p $O
export TMPDIR=/tmp
bash scripts/gpu_tests.sh > $O/gpu_tests_summary.txt 2>&1; rc=$?
cp gpurun_out/gpu_tests.log gpurun_out/smoke.log $O/ 2>/dev/null
tail -4 $O/gpu_tests_summary.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for WL in 4k_p8 4k_p8_mixed; do for L in libsvtme_base libsvtme; do
  SVTME_LIB=svt-av1-mirror_amd/$L.so timeout -k 10 200 python3 bench.py --workload $WL --steps 50 --warmup 10 --no-cpu-baseline --band-steps 0 --no-upload > $O/b_${L}_${WL}_r$r.json 2> $O/b_${L}_${WL}_r$r.err || { tail $O/b_${L}_${WL}_r$r.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1].split('/')[-1], round(d['value']/1e6,2), {k: v['avg_ms'] for k, v in r['stages'].items()})" $O/b_${L}_${WL}_r$r.json
done; done; done
timeout -k 10 600 python3 scripts/glue_rate.py $O/glue_rate.json 4k_p8_64f > $O/glue_rate.log 2>&1 || { tail -20 $O/glue_rate.log; exit 1; }
cut -c1-700 $O/glue_rate.log
