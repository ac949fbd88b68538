# round 4: the default bench line (realistic distances in the pipelined and band legs), the upload
# probe, and the 4K p8 profile with only the headline's launches traced (no band / SB-result legs)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python3 scripts/upload_probe.py 40 > $O/upload_probe.json 2> $O/upload_probe.err || { tail -20 $O/upload_probe.err; exit 1; }
cat $O/upload_probe.json
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('default', d['value'], d['roofline']['frac'], d['roofline']['chip'], d['upload'], d['band_8k'])" $O/bench_default.json
WL=4k_p8 TAG=r04k/r04_4k_p8 bash scripts/gpu_profile.sh > $O/prof_4k_p8.log 2>&1 || { tail -20 $O/prof_4k_p8.log; exit 1; }
tail -1 $O/prof_4k_p8.log
python3 -c "import json; d=json.load(open('$O/r04_4k_p8/pmc_summary.json')); c=d['counters_avg_per_launch']; print(d['hbm_bytes_per_launch'], c['SQ_WAIT_ANY']/c['SQ_WAVE_CYCLES'], c['TA_ADDR_STALLED_BY_TC_CYCLES_sum'])"
