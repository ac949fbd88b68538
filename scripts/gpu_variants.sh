# bench sweep of library variants (SVTME_LIB): usage VARIANTS="A B C" bash scripts/gpu_variants.sh
cd "$GRAFT_REPO_ROOT"
for v in ${VARIANTS:-A}; do
  SVTME_LIB=$GRAFT_REPO_ROOT/svt-av1-mirror_amd/libsvtme_v$v.so WLS="${WLS:-4k_p8}" PICS="${PICS:-1 4}" TAG=var_$v bash scripts/gpu_sweep.sh || exit 1
done
