# VALU / SALU / LDS instruction counts of the k_hme stop-after builds (scripts/build_phase_libs.sh):
# the differences between consecutive builds are the phases' instruction counts.
# usage: WL=4k_p8 P=1 [PMC="SQ_... TA_..."] [O=${O:-gpurun_out/phase_pmc}] bash scripts/gpu_phase_pmc.sh
# then: python3 scripts/phase_pmc_summary.py $O (per-SB counts per phase, JSON)
cd "$GRAFT_REPO_ROOT"
WL=${WL:-4k_p8}; P=${P:-1}
O=${O:-gpurun_out/phase_pmc}
mkdir -p $O
export TMPDIR=/tmp
for k in ${KS:-1 2 3 4 5 55 6 full}; do
  lib=svt-av1-mirror_amd/libsvtme_stop$k.so
  [ "$k" = full ] && lib=svt-av1-mirror_amd/libsvtme.so
  SVTME_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "k_hme" \
    --pmc ${PMC:-SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES} \
    -d "$GRAFT_REPO_ROOT/$O/stop$k" -o run --output-format csv -- python3 scripts/phase_cost.py $WL $P stop_after_$k > $O/stop$k.log 2>&1 || { echo "stop$k failed"; tail -5 $O/stop$k.log; exit 1; }
  echo "stop$k done"
done
