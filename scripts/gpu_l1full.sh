# k_l1_full bring-up: MCTF parity + golden TF cases + the TF-level encodes, then the TF-ME bench
# with and without it (SVTME_NO_L0_FULL=1: k_stage_a; the A/B variable is the last kernel brought up)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/l1full; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 120 python3 -u -m pytest tests/test_gpu_parity.py -k mctf -x -v -m gpu --timeout 60 --timeout-method thread > $O/mctf.log 2>&1 || { tail -30 $O/mctf.log; exit 1; }
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_encoder.py -k "mctf or tf or golden or 360p_p8 or ra360 or 1080p_p8 or 240p" -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -12; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in 0 1; do
  if [ $v = 1 ]; then export SVTME_NO_L0_FULL=1; else unset SVTME_NO_L0_FULL; fi
  timeout -k 10 200 python3 bench.py --workload 4k_tf_p8 --steps 20 --warmup 5 --no-cpu-baseline --band-steps 0 > $O/b_v${v}_r$r.json 2> $O/b_v${v}_r$r.err || { tail $O/b_v${v}_r$r.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], {k: v['avg_ms'] for k, v in r['stages'].items()}, r['valu_sad']['frac'])" $O/b_v${v}_r$r.json
done; done
