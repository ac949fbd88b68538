cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${R:-r06l} ROUNDS=3 bash scripts/gpu_ab_tests.sh || exit 1
O=gpurun_out/${R:-r06l}/stamps bash scripts/gpu_stamps.sh
