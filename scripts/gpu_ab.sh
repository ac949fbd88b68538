# zero-copy through a few streaming workgroups: pyramid equality, upload legs, GPU suite, served rate
export TMPDIR=/tmp; O=gpurun_out/r05x; mkdir -p $O
timeout -k 10 120 python3 -u scripts/zero_copy_probe.py > $O/zc.json 2> $O/zc.err || { tail -20 $O/zc.err; exit 1; }
cat $O/zc.json
timeout -k 10 900 python3 -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/t.log 2>&1; rc=$?; tail -1 $O/t.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/t.log | head; exit $rc; }
for r in 1 2; do
timeout -k 10 300 python3 -u bench.py --band-steps 0 --steady-steps 0 > $O/bench$r.json 2> $O/bench$r.err || { tail -20 $O/bench$r.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench$r.json')); u=d['upload']; print(d['value'], u['pinned_ms_per_picture'], u['pipelined_ms_per_picture'], u['async_upload_only_ms_per_picture'], u['pcie_inclusive_sb_per_s'], u['pipelined_sb_per_s'], d['cpu_baseline']['value'])"
done
GLUE_RATE_REPEAT=2 timeout -k 10 300 python3 -u scripts/glue_rate.py $O/glue.json 4k_p8_64f > $O/glue.log 2>&1 || { tail -20 $O/glue.log; exit 1; }
python3 -c "import json; [print({k: d.get(k) for k in ('identical','served_sb_per_s','max_job_ms','upload_ms')}) for d in json.load(open('$O/glue.json'))]"
