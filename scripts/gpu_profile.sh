# bench one workload + rocprofv3 kernel trace + PMC passes (each pass its own run)
# usage: WL=4k_p8 TAG=r02_4k_p8 bash scripts/gpu_profile.sh
# (the kernel-trace and PMC passes run one submission lane: kernel durations without overlap)
cd "$GRAFT_REPO_ROOT"
WL=${WL:-4k_p8}; TAG=${TAG:-prof_$WL}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
{ echo "nproc $(nproc)"; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())";
  cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo; } > $O/host.txt 2>&1
timeout -k 10 300 python3 -u bench.py --workload $WL --steps 50 --warmup 10 ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/kt" -o run --output-format csv -- python3 bench.py --workload $WL --steps 50 --warmup 10 --no-cpu-baseline --no-single-picture --no-upload --no-records-only --band-steps 0 --lanes 1 > $O/kt.log 2>&1 || { echo "rocprof kt failed"; tail -20 $O/kt.log; exit 1; }
run_pass() {
  name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "k_stage|k_hme|k_fp|k_l0|k_l1" --pmc "$@" -d "$GRAFT_REPO_ROOT/$O/pmc_$name" -o run --output-format csv -- python3 bench.py --workload $WL --steps 5 --warmup 2 --no-cpu-baseline --no-single-picture --no-upload --no-records-only --band-steps 0 --lanes 1 > $O/pmc_$name.log 2>&1 || { echo "pass $name failed $?"; tail -20 $O/pmc_$name.log; return 1; }
}
run_pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU && \
run_pass sq2 SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH && \
run_pass fetch FETCH_SIZE && \
run_pass write WRITE_SIZE && \
run_pass sq3 SQ_INST_CYCLES_VMEM_RD SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM SQ_WAIT_INST_LDS SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL && \
run_pass ta TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum && \
python3 scripts/pmc_summary.py $O > /dev/null && echo "profile done: $O"
