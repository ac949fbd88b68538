# closing check of a round: smoke + the whole -m gpu suite, three driver-style bench lines
# (fresh processes, the defaults = --steps 20 --warmup 5) and one 64-frame 4K encode's served rate
# usage: [O=gpurun_out/closing] bash scripts/gpu_closing.sh
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${O:-gpurun_out/closing}; mkdir -p $O
bash scripts/gpu_tests.sh > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
cp gpurun_out/gpu_tests.log gpurun_out/smoke.log $O/ 2>/dev/null
for r in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py > $O/bench$r.json 2> $O/bench$r.err || { tail -20 $O/bench$r.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); u=d['upload']; r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r['traffic'], (d.get('steady_state') or {}).get('value'), u['pipelined_sb_per_s'], u['pcie_inclusive_sb_per_s'], d['cpu_baseline']['value'], d['parity_vs_cpu'])" $O/bench$r.json
done
timeout -k 10 300 python3 -u scripts/glue_rate.py $O/glue.json 4k_p8_64f > $O/glue.log 2>&1 || { tail -20 $O/glue.log; exit 1; }
python3 -c "import json; [print({k: d.get(k) for k in ('identical','served_sb_per_s','job_latency_ms','max_job_ms','prefetched','prefetch_hits','unused_jobs')}) for d in json.load(open('$O/glue.json'))]"
