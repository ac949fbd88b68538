# one iteration: GPU tests, A/B of the working tree against libsvtme_prev.so (4K p8, then
# WL2 if set), k_hme phase stamps.  usage: R=tag [WL2=1080p_sa64] bash scripts/gpu_iter.sh
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${R:-iter} ROUNDS=3 bash scripts/gpu_ab_tests.sh || exit 1
if [ -n "${WL2:-}" ]; then LIBS=prev WL=$WL2 ROUNDS=2 O=gpurun_out/${R:-iter}/ab_$WL2 bash scripts/gpu_ab_bench.sh || exit 1; fi
O=gpurun_out/${R:-iter}/stamps bash scripts/gpu_stamps.sh
