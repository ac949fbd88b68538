# bench sweep over pictures per step (batched launches), no CPU leg
# usage: WLS="4k_p8 1080p_sa64" PICS="1 2 4 8" TAG=sweep bash scripts/gpu_sweep.sh
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-sweep}
O=gpurun_out/$TAG
mkdir -p $O
for wl in ${WLS:-4k_p8}; do
  for p in ${PICS:-1 2 4 8}; do
    timeout -k 10 120 python3 -u bench.py --workload $wl --pictures $p --steps ${STEPS:-50} --warmup 10 --no-cpu-baseline \
      > $O/${wl}_p$p.json 2> $O/${wl}_p$p.err || { echo "bench $wl p$p failed $?"; tail -20 $O/${wl}_p$p.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/${wl}_p$p.json')); r=d['roofline']; print('$wl', $p, d['value'], d['ms_per_step'], r['frac'], {k: v['avg_ms'] for k, v in r['stages'].items()})"
  done
done
