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
# this round's build on every BASELINE workload (50 steps, CPU baseline + parity check each)
for WL in 4k_p8_mixed 8k_p8 1080p_sa64 4k10_p6 4k_tf_p8 1080p_p8; do
  timeout -k 10 300 python3 bench.py --workload $WL --steps 50 --warmup 10 --band-steps 0 > $O/bench_$WL.json 2> $O/bench_$WL.err || { tail -20 $O/bench_$WL.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], r['frac'], r['valu_sad']['frac'], {k: v['avg_ms'] for k, v in r['stages'].items()}, d['parity_vs_cpu'], d['cpu_baseline']['value'])" $O/bench_$WL.json
done
