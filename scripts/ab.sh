# A/B timing of two library builds in one GPU session, interleaved:
# usage: A=svt-av1-mirror_amd/libsvtme_base.so B=svt-av1-mirror_amd/libsvtme.so bash scripts/ab.sh
cd "$GRAFT_REPO_ROOT"
for r in 1 2 3; do
  for L in "$A" "$B"; do
    for P in 1 4; do
      SVTME_LIB=$L timeout -k 10 100 python3 scripts/phase_cost.py ${WL:-4k_p8} $P $(basename $L .so) || exit 1
    done
  done
done
