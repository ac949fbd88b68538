# SQ instruction / stall counters for k_me_sb (separate --pmc passes, kernel trace only)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
run_pass() {
  name=$1; shift
  timeout -k 10 600 rocprofv3 --kernel-trace --kernel-include-regex "k_me_sb|k_stage" --pmc "$@" -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$name" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --kernel-samples 2 ${BENCH_ARGS} > gpurun_out/pmc_$name.log 2>&1 || { echo "pass $name failed $?"; tail -20 gpurun_out/pmc_$name.log; return 1; }
}
run_pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU && \
run_pass sq2 SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH && \
run_pass fetch FETCH_SIZE && \
run_pass write WRITE_SIZE && \
python3 scripts/pmc_summary.py gpurun_out
