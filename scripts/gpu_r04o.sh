# k_fp_wide quantisation probe: the 1080p 64x64 override with 2..10 pictures per launch (1 020
# workgroups per picture over 1 280 resident slots): time per picture of k_fp_wide and of the step
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04o; mkdir -p $O; export TMPDIR=/tmp
for P in 2 3 4 5 6 8 10; do
  timeout -k 10 200 python3 bench.py --workload 1080p_sa64 --pictures $P --steps 40 --warmup 8 --no-cpu-baseline --band-steps 0 --no-upload --no-single-picture --no-sb-results > $O/b_p$P.json 2> $O/b_p$P.err || { tail $O/b_p$P.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; P=int(sys.argv[2]); print('P', P, 'M SB/s', round(d['value']/1e6,3), 'valu_sad', r['valu_sad']['frac'], 'fp_wide ms/pic', round(r['stages']['k_fp_wide']['avg_ms']/P,4), 'step ms/pic', round(d['ms_per_step']/P,4))" $O/b_p$P.json $P
done
