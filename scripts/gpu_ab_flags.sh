# compiler scheduling flags A/B (libsvtme_f3: metric bias 0, f4: bias 100, f5: relaxed occupancy) vs the product
export TMPDIR=/tmp; O=gpurun_out/r05dd; mkdir -p $O
for r in 1 2 3; do for L in libsvtme libsvtme_f3 libsvtme_f4 libsvtme_f5; do
  SVTME_LIB=svt-av1-mirror_amd/$L.so timeout -k 10 100 python3 scripts/phase_cost.py 4k_p8 4 $L 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || exit 1
  SVTME_LIB=svt-av1-mirror_amd/$L.so timeout -k 10 100 python3 scripts/phase_cost.py 1080p_sa64 4 $L 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || exit 1
done; done
cat $O/ab.txt
