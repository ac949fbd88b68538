cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06b; mkdir -p $O
bash scripts/gpu_tests.sh > $O/tests.txt 2>&1 || { cat $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
for r in 1 2; do
  timeout -k 10 200 python3 -u bench.py --no-upload --band-steps 0 --no-cpu-baseline > $O/new_$r.json 2>> $O/b.err || exit 1
  SVTME_LIB=svt-av1-mirror_amd/libsvtme_base.so timeout -k 10 200 python3 -u bench.py --no-upload --band-steps 0 --no-cpu-baseline > $O/base_$r.json 2>> $O/b.err || exit 1
done
timeout -k 10 300 python3 -u bench.py > $O/full.json 2>> $O/b.err || exit 1
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-upload --band-steps 0 --workload 4k10_p6 > $O/p6.json 2>> $O/b.err || exit 1
for f in $O/*.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'], (d.get('records_only') or {}).get('value'), (d.get('steady_state') or {}).get('value'), d['roofline']['frac'], d.get('parity_vs_cpu'))" $f; done
