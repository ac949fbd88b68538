# Build a diagnostic variant of the product library (container; the GPU box runs it
# through SVTME_LIB): svt-av1-mirror_amd/libsvtme_<name>.so from the working tree.
# svtme_stages.hip is compiled with csrc/diag/svtme_diag.h force-included (the
# product build never includes it) and the extra defines; the other sources as the
# product build compiles them.
# usage: bash scripts/build_diag_lib.sh NAME [-DFLAG[=V] ...]
#   clk   -DSVTME_CLOCKBINS        in-kernel clock over time (scripts/clock_probe.py)
#   stamp -DSVTME_STAMPS           per-phase shader-clock stamps (scripts/hme_stamps.py)
#   stopK -DSVTME_STOP_AFTER=K     k_hme ends after phase K (scripts/gpu_phase_cost.sh)
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
C=svt-av1-mirror_amd/csrc
T=$(mktemp -d)
trap 'rm -rf "$T"' EXIT
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall"
/opt/rocm/bin/hipcc $FL -include $C/diag/svtme_diag.h "$@" -c -o $T/stages.o $C/svtme_stages.hip
for f in svtme_pyramid.hip svtme_pack.hip svtme_rtcd.hip svtme_host.cpp; do
  /opt/rocm/bin/hipcc $FL -c -o $T/$f.o $C/$f
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o svt-av1-mirror_amd/libsvtme_$NAME.so $T/*.o
echo "built svt-av1-mirror_amd/libsvtme_$NAME.so ($*)"
