# Build a diagnostic variant of the product library (container; the GPU box runs it
# through SVTME_LIB): svt-av1-mirror_amd/libsvtme_<name>.so from the working tree
# with extra defines.
# usage: bash scripts/build_diag_lib.sh NAME [-DFLAG[=V] ...]
#   clk   -DSVTME_CLOCKBINS        in-kernel clock over time (scripts/clock_probe.py)
#   stamp -DSVTME_STAMPS           per-phase shader-clock stamps (scripts/hme_stamps.py)
#   stopK -DSVTME_STOP_AFTER=K     k_hme ends after phase K (scripts/gpu_phase_cost.sh)
#   diag  -DSVTME_DIAG_A1=1|2, -DSVTME_DIAG_NO_L1_PREHME  A1 load / list-1 pre-HME cost probes (wrong results)
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall "$@" \
  -o svt-av1-mirror_amd/libsvtme_$NAME.so svt-av1-mirror_amd/csrc/svtme_pyramid.hip svt-av1-mirror_amd/csrc/svtme_pack.hip \
  svt-av1-mirror_amd/csrc/svtme_stages.hip svt-av1-mirror_amd/csrc/svtme_rtcd.hip svt-av1-mirror_amd/csrc/svtme_host.cpp
echo "built svt-av1-mirror_amd/libsvtme_$NAME.so ($*)"
