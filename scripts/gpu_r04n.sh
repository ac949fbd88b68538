# round 4: svtme_reserve (glue: no device allocation on the first jobs) -- packed-output tests,
# encoder bitstreams + glue rate; then the 1080p 64x64 override profile (kernel trace + PMC passes)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04n; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_pack.py tests/test_encoder.py -m gpu -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python3 scripts/glue_rate.py $O/glue_rate.json 4k_p8_64f 4k_p8_16f 1080p_p8 > $O/glue_rate.log 2>&1 || { tail -20 $O/glue_rate.log; exit 1; }
cut -c1-200 $O/glue_rate.log
WL=1080p_sa64 TAG=r04n/r04_1080p_sa64 bash scripts/gpu_profile.sh > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
tail -1 $O/prof.log
