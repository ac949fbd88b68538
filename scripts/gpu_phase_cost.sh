# Phase throughput costs of k_hme: builds (in the container, scripts/build_phase_libs.sh)
# that end after stamp k; run each on the GPU box, one process per build.
# usage: WL=4k_p8 P=4 bash scripts/gpu_phase_cost.sh
cd "$GRAFT_REPO_ROOT"
WL=${WL:-4k_p8}; P=${P:-4}
mkdir -p gpurun_out
for k in ${KS:-1 2 3 4 5 55 6 full}; do
  lib=svt-av1-mirror_amd/libsvtme_stop$k.so
  [ "$k" = full ] && lib=svt-av1-mirror_amd/libsvtme.so
  SVTME_LIB=$lib timeout -k 10 120 python3 scripts/phase_cost.py $WL $P stop_after_$k || exit 1
done
