export TMPDIR=/tmp; O=gpurun_out/r05p; mkdir -p $O
timeout -k 10 200 python3 -u scripts/glue_rate.py $O/glue.json 4k_p8_64f > $O/glue.log 2>&1 || { tail -20 $O/glue.log; exit 1; }
python3 - <<'PY'
import json
d=json.load(open('gpurun_out/r05p/glue.json'))[0]
print({k: d.get(k) for k in ('identical','served_sb_per_s','submit_ms','launches')})
for j in d['jobs']:
    if j['tf']==1 or j['done_ms']-j['create_ms']>0.2:
        print(j['pn'], j['tf'], 'prep', j.get('prep_ms'), 'lock', j.get('lock_ms'), 'sub', round(j['submitted_ms']-j['create_ms'],3), 'tot', round(j['done_ms']-j['create_ms'],3), 'gpu', j['gpu_ms'], 'copy', j['copy_ms'])
PY
