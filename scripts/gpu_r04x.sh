# round 4: picture release without a device-wide wait (deferred free / same-size reuse) -- the whole
# GPU suite, glue rate, and a 64-frame encode with at most 12 resident pictures (evictions)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04x; mkdir -p $O; export TMPDIR=/tmp
bash scripts/gpu_tests.sh > $O/gpu_tests_summary.txt 2>&1; rc=$?
cp gpurun_out/gpu_tests.log $O/ 2>/dev/null
tail -4 $O/gpu_tests_summary.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 scripts/glue_rate.py $O/glue_rate.json 4k_p8_64f 4k_p8_16f > $O/glue_rate.log 2>&1 || { tail -20 $O/glue_rate.log; exit 1; }
cut -c1-160 $O/glue_rate.log
SVTME_GLUE_RESIDENT=12 timeout -k 10 600 python3 scripts/glue_rate.py $O/glue_rate_resident12.json 4k_p8_64f > $O/glue_rate_resident12.log 2>&1 || { tail -20 $O/glue_rate_resident12.log; exit 1; }
python3 -c "
import json
for c in json.load(open('$O/glue_rate_resident12.json')):
    print(c['case'], c['identical'], 'evictions', c['evictions'], 'served M', round(c['served_sb_per_s']/1e6, 2), 'uploads', c['uploads'])
"
