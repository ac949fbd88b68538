# Device assembly of every HIP source: fail if any scalar-cache write form appears
# (s_store*, s_buffer_store*, s_scratch_store*, scalar atomics, s_dcache_wb/discard).
set -e
cd "$(dirname "$0")/../svt-av1-mirror_amd/csrc"
mkdir -p /tmp/svtme_isa
bad=0
for f in *.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S "$f" -o "/tmp/svtme_isa/${f%.hip}.s"
  n=$(grep -cE "^\s*(s_store|s_buffer_store|s_scratch_store|s_atomic|s_buffer_atomic|s_dcache_wb|s_dcache_discard)" "/tmp/svtme_isa/${f%.hip}.s" || true)
  echo "$f: $n scalar-write instructions"
  [ "$n" = "0" ] || bad=1
done
exit $bad
