# container: the SVTME_STOP_AFTER=k diagnostic builds used by scripts/gpu_phase_cost.sh
cd "$(dirname "$0")/.."
for k in 1 2 3 4 5 55 6; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DSVTME_STOP_AFTER=$k \
    -o svt-av1-mirror_amd/libsvtme_stop$k.so svt-av1-mirror_amd/csrc/*.hip svt-av1-mirror_amd/csrc/svtme_host.cpp &
done
wait
