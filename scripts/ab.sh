# A/B timing of library builds in one GPU session, interleaved (3 rounds, 1 and 4 pictures per launch):
# usage: LIBS="svt-av1-mirror_amd/libsvtme_a.so svt-av1-mirror_amd/libsvtme_b.so" bash scripts/ab.sh
#        (or A=... B=... as before); WL picks the workload (default 4k_p8)
cd "$GRAFT_REPO_ROOT"
LIBS=${LIBS:-"$A $B"}
for r in 1 2 3; do
  for L in $LIBS; do
    for P in ${PICS:-1 4}; do
      SVTME_LIB=$L timeout -k 10 100 python3 scripts/phase_cost.py ${WL:-4k_p8} $P $(basename $L .so) || exit 1
    done
  done
done
