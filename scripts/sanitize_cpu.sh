#!/bin/bash
# The CPU-side code of this repository under AddressSanitizer + UndefinedBehaviorSanitizer
# (build container only; the reference's CI does the same for its encoder,
# .gitlab/workflows/linux/.gitlab-ci.yml:219-249):
#   build/asan/liboracle.so        oracle/svtme_oracle.c + svtme_oracle_kernels.c
#   build/asan/libsvtme_synth.so   svt-av1-mirror_amd/csrc/synth.c
#   build/asan/liboraclejob.so     oracle/svtme_oraclejob.c (+ the oracle)
#   build/asan/svtav1enc_ora       the reference encoder + integration/svtme_svt_glue.c
#                                  (glue and job backend instrumented)
# then the whole CPU suite (pytest -m "not gpu") loads them instead of the
# regular builds (SVTME_ORACLE_LIB, SVTME_SYNTH_LIB, SVTME_ENC_DIR).
# Usage: bash scripts/sanitize_cpu.sh [extra pytest args]
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$ROOT/build/asan"
REF=/root/reference
mkdir -p "$OUT"
SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g -O1"

gcc $SAN -std=c11 -fPIC -shared -Wall -Wextra -Wno-unused-parameter -o "$OUT/liboracle.so" \
    "$ROOT/oracle/svtme_oracle.c" "$ROOT/oracle/svtme_oracle_kernels.c" -lpthread
gcc $SAN -fPIC -shared -o "$OUT/libsvtme_synth.so" "$ROOT/svt-av1-mirror_amd/csrc/synth.c"
gcc $SAN -std=gnu11 -fPIC -shared -Wall -Wextra -Wno-unused-parameter -o "$OUT/liboraclejob.so" \
    "$ROOT/oracle/svtme_oraclejob.c" "$ROOT/oracle/svtme_oracle.c" "$ROOT/oracle/svtme_oracle_kernels.c" -lpthread

ENC="$ROOT/oracle/_ref/enc"
if [ -d "$REF/Source" ]; then
    make -s -C "$ROOT/oracle" -f encoder.mk -j8 _ref/enc/svtav1enc _ref/enc/libsvtenc.a
    INC="-I$REF -I$REF/Source/API -I$REF/Source/Lib/Codec -I$REF/Source/Lib/C_DEFAULT -I$REF/Source/Lib/Globals \
         -I$REF/third_party/fastfeat -I$ENC/gen -I$ROOT/include"
    gcc $SAN -std=gnu99 -fPIC -ffunction-sections -DSVTME_GLUE_WRAP -DEXCLUDE_HASH=0 -DREPRODUCIBLE_BUILDS=0 \
        -DEN_AVX512_SUPPORT=0 -DHAVE_CPUINFO=0 -DNDEBUG $INC -c -o "$OUT/glue.o" "$ROOT/integration/svtme_svt_glue.c"
    # (the wraps of oracle/encoder.mk's WRAP)
    gcc -fsanitize=address,undefined -o "$OUT/svtav1enc_ora" "$ENC"/obj/Source/App/*.o \
        "$ENC"/obj/third_party/safestringlib/*.o "$OUT/glue.o" "$ENC/libsvtenc.a" \
        -Wl,--wrap=svt_aom_motion_estimation_b64 -Wl,--wrap=svt_aom_downsample_filtering_input_picture \
        -Wl,--wrap=svt_av1_enc_deinit -Wl,--wrap=svt_av1_enc_init \
        -Wl,--wrap=svt_post_full_object \
        -L"$OUT" -loraclejob -Wl,-rpath,"$OUT" -Wl,--gc-sections -lpthread -lm
fi

# python is not instrumented: the runtimes are preloaded (ahead of anything already preloaded)
ASAN_RT="$(gcc -print-file-name=libasan.so)"
UBSAN_RT="$(gcc -print-file-name=libubsan.so)"
cd "$ROOT"
SVTME_ORACLE_LIB="$OUT/liboracle.so" SVTME_SYNTH_LIB="$OUT/libsvtme_synth.so" SVTME_ENC_DIR="$OUT" \
ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
LD_PRELOAD="$ASAN_RT $UBSAN_RT${LD_PRELOAD:+ $LD_PRELOAD}" \
    python -m pytest tests -x -q -m "not gpu" -p no:cacheprovider "$@"
