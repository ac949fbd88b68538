# round 4: glue start-up (registration and pool fill outside the job locks): encoder bitstreams + glue rate;
# then the k_fp_wide quantisation probe
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04p; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_encoder.py tests/test_pack.py -m gpu -q --timeout 150 --timeout-method thread > $O/enc.log 2>&1 || { tail -30 $O/enc.log; exit 1; }
tail -1 $O/enc.log
timeout -k 10 600 python3 scripts/glue_rate.py $O/glue_rate.json 4k_p8_64f 4k_p8_16f 1080p_p8 > $O/glue_rate.log 2>&1 || { tail -20 $O/glue_rate.log; exit 1; }
cut -c1-200 $O/glue_rate.log
bash scripts/gpu_r04o.sh
