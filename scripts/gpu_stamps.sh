# per-phase k_hme latency from the stamps build (scripts/build_diag_lib.sh stamp -DSVTME_STAMPS)
cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/stamps}; mkdir -p $O
for WL in ${WLS:-4k_p8}; do
  for P in ${PICS:-4}; do
    timeout -k 10 120 python3 -u scripts/hme_stamps.py $WL $P ${MODE:-} > $O/stamps_${WL}_x$P${MODE:+_$MODE}.txt 2>&1 || { tail -20 $O/stamps_${WL}_x$P${MODE:+_$MODE}.txt; exit 1; }
    cat $O/stamps_${WL}_x$P${MODE:+_$MODE}.txt
  done
done
