# k_hme A1 tile height (HT16) A/B: 3 (product) vs 2 vs 4 -- parity per library, then 4K p8 and mixed,
# 3 interleaved rounds
cd "$GRAFT_REPO_ROOT"

LIBS="libsvtme libsvtme_ht2 libsvtme_ht4" WLS="4k_p8 4k_p8_mixed" ROUNDS=3 STEPS=50 bash scripts/gpu_ab_libs.sh
