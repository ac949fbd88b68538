# A/B of library builds in fresh processes at the driver's window (bench.py defaults, no CPU leg):
# value, records_only, steady (whole / records-only) of each, 2 interleaved rounds.
# usage: LIBS="prev" [WL=4k_p8] [ROUNDS=2] bash scripts/gpu_ab_bench.sh   (the working-tree libsvtme.so runs as "cur")
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${O:-gpurun_out/ab}; mkdir -p $O
A="--no-upload --band-steps 0 --no-cpu-baseline --workload ${WL:-4k_p8} ${BENCH_ARGS:-}"
for r in $(seq 1 ${ROUNDS:-2}); do
  timeout -k 10 200 python3 -u bench.py $A > $O/cur_$r.json 2>> $O/err || exit 1
  for L in ${LIBS:-}; do
    SVTME_LIB=svt-av1-mirror_amd/libsvtme_$L.so timeout -k 10 200 python3 -u bench.py $A > $O/${L}_$r.json 2>> $O/err || exit 1
  done
done
for f in $O/*.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d.get('steady_state') or {}; print(sys.argv[1], d['value'], d['ms_per_step'], (d.get('records_only') or {}).get('value'), s.get('value'), (s.get('records_only') or {}).get('value'), d['roofline']['frac'], {k: v['avg_ms'] for k, v in d['roofline']['stages'].items()})" $f; done
