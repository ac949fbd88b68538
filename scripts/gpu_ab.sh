export TMPDIR=/tmp; O=gpurun_out/r05i; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_configs.py tests/test_gpu_parity.py tests/test_gpu_fpwide.py tests/test_pack.py > $O/t.log 2>&1; echo "t rc=$?"; tail -2 $O/t.log
for r in 1 2 3; do for L in libsvtme_base libsvtme_v1 libsvtme_v2; do
  SVTME_LIB=svt-av1-mirror_amd/$L.so timeout -k 10 100 python3 scripts/phase_cost.py 4k_p8 4 $L >> $O/ab.txt 2>&1 || exit 1
  SVTME_LIB=svt-av1-mirror_amd/$L.so timeout -k 10 100 python3 scripts/phase_cost.py 4k_p8_mixed 4 $L >> $O/ab.txt 2>&1 || exit 1
done; done
SVTME_LIB=svt-av1-mirror_amd/libsvtme_stamp.so timeout -k 10 100 python3 scripts/hme_stamps.py 4k_p8 4 > $O/stamps.json 2>&1 || exit 1
cat $O/ab.txt
