# whole 4K p8 encodes through the glue (scripts/glue_rate.py): served rate, upload calls, bitstreams
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${O:-gpurun_out/glue}; mkdir -p $O
GLUE_RATE_REPEAT=${REPS:-2} timeout -k 10 600 python3 -u scripts/glue_rate.py $O/glue.json ${CASES:-4k_p8_64f} > $O/glue.log 2>&1 || { tail -30 $O/glue.log; exit 1; }
grep -v "^ " $O/glue.log | python3 -c "
import json, sys
for line in sys.stdin:
    line = line.strip()
    if not line.startswith('{'):
        continue
    r = json.loads(line)
    print(r['case'], 'identical', r['identical'], 'served', round(r['served_sb_per_s'] / 1e6, 2), 'M SB/s; with uploads',
          round(r['served_sb_per_s_with_uploads'] / 1e6, 2), '; uploads', r['uploads'], 'eager_upload_ms', r['eager_upload_ms'],
          'per upload', round(r['eager_upload_ms'] / max(1, r['uploads']), 4), 'init_registrations', r.get('init_registrations'),
          'registrations', r['registrations'], 'register_ms', r['register_ms'], 'max_job_ms', r['max_job_ms'], 'upload calls', r.get('upload_call_ms'))
"
