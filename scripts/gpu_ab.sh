# glue prefetch: GPU encoder tests, then served rate over 64-frame 4K encodes with and without it
export TMPDIR=/tmp; O=gpurun_out/r05n; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_encoder.py > $O/t.log 2>&1; rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || exit $rc
GLUE_RATE_REPEAT=3 timeout -k 10 300 python3 -u scripts/glue_rate.py $O/glue_prefetch.json 4k_p8_64f > $O/glue_prefetch.log 2>&1 || { tail -20 $O/glue_prefetch.log; exit 1; }
SVTME_GLUE_PREFETCH=0 timeout -k 10 200 python3 -u scripts/glue_rate.py $O/glue_noprefetch.json 4k_p8_64f > $O/glue_noprefetch.log 2>&1 || { tail -20 $O/glue_noprefetch.log; exit 1; }
python3 - <<'PY'
import json
for f in ['gpurun_out/r05n/glue_prefetch.json','gpurun_out/r05n/glue_noprefetch.json']:
    for d in json.load(open(f)):
        print(f.split('/')[-1], {k: d.get(k) for k in ('identical','served_sb_per_s','job_latency_ms','busy_ms','wait_ms','prefetched','prefetch_hits','prefetch_ready','unused_jobs','max_job_ms','max_inflight','gpu_encoder_seconds')})
PY
