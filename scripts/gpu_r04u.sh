# round 4: glue rate with the prefill timed apart
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04u; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python3 scripts/glue_rate.py $O/glue_rate.json 4k_p8_64f 4k_p8_16f 1080p_p8 > $O/glue_rate.log 2>&1 || { tail -20 $O/glue_rate.log; exit 1; }
python3 -c "
import json
for c in json.load(open('$O/glue_rate.json')):
    print(c['case'], c['identical'], round(c['served_sb_per_s']/1e6,2), round(c['served_sb_per_s_with_uploads']/1e6,2), c['busy_ms'], c['eager_upload_ms'], c["prefill_ms"], c["registrations"], c["register_ms"], c["uploads"], c['unpinned_uploads'])
"
