# Build libsvtme_<name>.so from the product sources with FILES (default
# svtme_stages.hip) taken from git revision REV (default HEAD) -- the "A" side of
# an A/B against the working tree.
# usage: REV=HEAD NAME=base [FILES="svtme_host.cpp"] [SED='s/#define HT16 3/#define HT16 4/'] bash scripts/build_ab_lib.sh
# (SED: a sed expression applied to the copy of svtme_stages.hip, for one-constant experiments)
set -e
cd "$(dirname "$0")/.."
REV=${REV:-HEAD}; NAME=${NAME:-base}
T=svt-av1-mirror_amd/.ab_src_$NAME; rm -rf "$T"; mkdir -p "$T"  # two levels below the root: the sources include ../../include/svtme.h
cp svt-av1-mirror_amd/csrc/*.hip svt-av1-mirror_amd/csrc/*.cpp svt-av1-mirror_amd/csrc/*.h "$T"/
for f in ${FILES:-svtme_stages.hip}; do git show "$REV":svt-av1-mirror_amd/csrc/$f > "$T"/$f; done
if [ -n "${SED:-}" ]; then sed -i "$SED" "$T"/svtme_stages.hip; fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Iinclude \
  -o svt-av1-mirror_amd/libsvtme_$NAME.so "$T"/svtme_pyramid.hip "$T"/svtme_pack.hip "$T"/svtme_stages.hip \
  "$T"/svtme_rtcd.hip "$T"/svtme_host.cpp
rm -rf "$T"
echo "built svt-av1-mirror_amd/libsvtme_$NAME.so from $REV"
