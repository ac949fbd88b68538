# round 4: asynchronous uploads with the copy on its own stream (staging rotation) -- upload-related
# parity + encoder tests on the new library, then the upload A/B against HEAD's (libsvtme_up0)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04w; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_pack.py tests/test_encoder.py -m gpu -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do for L in libsvtme_up0 libsvtme; do
  SVTME_LIB=svt-av1-mirror_amd/$L.so timeout -k 10 120 python3 scripts/upload_probe.py 40 > $O/up_${L}_r$r.json 2> $O/up_${L}_r$r.err || { tail $O/up_${L}_r$r.err; exit 1; }
  echo "$L r$r $(cat $O/up_${L}_r$r.json)"
done; done
for r in 1 2; do for L in libsvtme_up0 libsvtme; do
  SVTME_LIB=svt-av1-mirror_amd/$L.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --band-steps 0 --no-single-picture --no-sb-results > $O/b_${L}_r$r.json 2> $O/b_${L}_r$r.err || { tail $O/b_${L}_r$r.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); u=d['upload']; print(sys.argv[1].split('/')[-1], round(d['value']/1e6,2), u['pinned_ms_per_picture'], u['pipelined_ms_per_picture'], u['async_upload_only_ms_per_picture'])" $O/b_${L}_r$r.json
done; done
