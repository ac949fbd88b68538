# Extra PMC passes on the default k_hme launch (4 pictures): instruction fetch,
# I-cache, scalar, L1->L2 latency. One pass per counter group, each under its own kill timeout.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmc_extra
mkdir -p $O
export TMPDIR=/tmp
pass() {
  name=$1; shift
  timeout -s KILL 60 rocprofv3 --kernel-trace --kernel-include-regex "k_hme" --pmc "$@" -d "$GRAFT_REPO_ROOT/$O/$name" \
    -o run --output-format csv -- python3 scripts/phase_cost.py 4k_p8 4 $name > $O/$name.log 2>&1 || { echo "pass $name failed"; tail -5 $O/$name.log; return 1; }
  echo "pass $name ok"
}
pass sq_fetch SQ_IFETCH SQ_IFETCH_LEVEL SQ_INST_CYCLES_SALU SQ_INST_CYCLES_SMEM SQ_INST_LEVEL_SMEM SQ_BUSY_CU_CYCLES SQ_WAVES SQ_WAVE_CYCLES && \
pass sqc_icache SQC_ICACHE_HITS SQC_ICACHE_MISSES && \
pass tcp_lat TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum
