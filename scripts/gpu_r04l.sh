# round 4: eager uploads (each picture uploaded when the encoder's analysis of it ends):
# encoder bitstream tests, glue rate with and without them
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04l; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_encoder.py -m gpu -q --timeout 150 --timeout-method thread > $O/enc_tests.log 2>&1 || { tail -30 $O/enc_tests.log; exit 1; }
tail -1 $O/enc_tests.log
timeout -k 10 600 python3 scripts/glue_rate.py $O/glue_rate.json 4k_p8_64f 4k_p8_16f 1080p_p8 > $O/glue_rate.log 2>&1 || { tail -20 $O/glue_rate.log; exit 1; }
cut -c1-1200 $O/glue_rate.log
SVTME_GLUE_EAGER=0 timeout -k 10 300 python3 scripts/glue_rate.py $O/glue_rate_job_time.json 4k_p8_64f > $O/glue_rate_job_time.log 2>&1 || { tail -20 $O/glue_rate_job_time.log; exit 1; }
cut -c1-1200 $O/glue_rate_job_time.log
