# round-3 profile of HEAD's k_hme at 4K p8: bench + kernel trace + PMC passes (gpu_profile.sh),
# the stop-after phase costs (4 pictures per launch) and the per-workgroup stamps
cd "$GRAFT_REPO_ROOT"
WL=4k_p8 TAG=r03_4k_p8 bash scripts/gpu_profile.sh || exit 1
WL=4k_p8 P=4 bash scripts/gpu_phase_cost.sh > gpurun_out/r03_4k_p8/phase_cost.txt 2>&1 || { echo "phase cost failed"; tail gpurun_out/r03_4k_p8/phase_cost.txt; exit 1; }
cat gpurun_out/r03_4k_p8/phase_cost.txt
SVTME_LIB=svt-av1-mirror_amd/libsvtme_stamp.so timeout -k 10 120 python3 scripts/hme_stamps.py 4k_p8 4 > gpurun_out/r03_4k_p8/stamps_x4.txt 2>&1 || { echo "stamps failed"; tail gpurun_out/r03_4k_p8/stamps_x4.txt; exit 1; }
head -12 gpurun_out/r03_4k_p8/stamps_x4.txt
