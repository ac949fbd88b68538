# A/B in fresh processes (the driver's window) of the whole output against the records alone and
# two diagnostic builds of finish_sb (no HBM stores / no candidate construction); 2 interleaved rounds
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${O:-gpurun_out/sbcost}; mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/rocprof_L.txt 2>&1 || true
A="--no-upload --band-steps 0 --no-cpu-baseline"
for r in 1 2; do
  timeout -k 10 200 python3 -u bench.py $A > $O/sb_$r.json 2>> $O/err || exit 1
  timeout -k 10 200 python3 -u bench.py $A --records-only > $O/ro_$r.json 2>> $O/err || exit 1
  for L in ${LIBS:-}; do
    SVTME_LIB=svt-av1-mirror_amd/libsvtme_$L.so timeout -k 10 200 python3 -u bench.py $A > $O/${L}_$r.json 2>> $O/err || exit 1
  done
done
for f in $O/*.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d.get('steady_state') or {}; print(sys.argv[1], d['value'], d['ms_per_step'], (d.get('records_only') or {}).get('value'), s.get('value'), (s.get('records_only') or {}).get('value'), d['roofline']['frac'], {k: v['avg_ms'] for k, v in d['roofline']['stages'].items()})" $f; done
