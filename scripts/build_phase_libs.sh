# container: the SVTME_STOP_AFTER=k diagnostic builds used by scripts/gpu_phase_cost.sh / gpu_phase_pmc.sh
cd "$(dirname "$0")/.."
for k in 1 2 3 4 5 55 6; do
  bash scripts/build_diag_lib.sh stop$k -DSVTME_STOP_AFTER=$k > /dev/null &
done
wait
ls svt-av1-mirror_amd/libsvtme_stop*.so
