# round 4: k_fp_wide row reads as ds_read_b64 (inline, explicit waits) -- parity of the product
# library, the 1080p 64x64 override A/B (fpw0: per-position 8x8 keys, fpw1: set minima with the
# compiler's ds_read2_b64, product: set minima + ds_read_b64), its profile; svtme_reserve: packed-output
# tests, encoder bitstreams + glue rate
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04n; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_configs.py tests/test_gpu_parity.py tests/test_pack.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do for L in libsvtme_fpw0 libsvtme_fpw1 libsvtme; do
  SVTME_LIB=svt-av1-mirror_amd/$L.so timeout -k 10 200 python3 bench.py --workload 1080p_sa64 --steps 50 --warmup 10 --no-cpu-baseline --band-steps 0 --no-upload > $O/b_${L}_r$r.json 2> $O/b_${L}_r$r.err || { tail $O/b_${L}_r$r.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1].split('/')[-1], round(d['value']/1e6,3), r['valu_sad']['frac'], {k: v['avg_ms'] for k, v in r['stages'].items()})" $O/b_${L}_r$r.json
done; done
WL=1080p_sa64 TAG=r04n/r04_1080p_sa64 bash scripts/gpu_profile.sh > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
tail -1 $O/prof.log
timeout -k 10 300 python3 -u -m pytest tests/test_encoder.py -m gpu -q --timeout 150 --timeout-method thread > $O/enc.log 2>&1 || { tail -30 $O/enc.log; exit 1; }
tail -1 $O/enc.log
timeout -k 10 600 python3 scripts/glue_rate.py $O/glue_rate.json 4k_p8_64f 4k_p8_16f 1080p_p8 > $O/glue_rate.log 2>&1 || { tail -20 $O/glue_rate.log; exit 1; }
cut -c1-200 $O/glue_rate.log
