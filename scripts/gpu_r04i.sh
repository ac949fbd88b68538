# round 4: encoder tests (bitstreams) + glue rate with cached page-locked encoder buffers, the N > 1
# rehearsal (2 ranks on the one GPU, gloo), then the 4K p8 profile of this round's kernels
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04i; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python3 -u -m pytest tests/test_encoder.py tests/test_pack.py -m gpu -q --timeout 150 --timeout-method thread > $O/enc_tests.log 2>&1 || { tail -30 $O/enc_tests.log; exit 1; }
tail -1 $O/enc_tests.log
timeout -k 10 600 python3 scripts/glue_rate.py $O/glue_rate.json 4k_p8_64f 4k_p8_16f 1080p_p8 > $O/glue_rate.log 2>&1 || { tail -20 $O/glue_rate.log; exit 1; }
cut -c1-900 $O/glue_rate.log
timeout -k 10 200 python3 scripts/band_probe.py > $O/band_probe.json 2> $O/band_probe.err || { tail -20 $O/band_probe.err; exit 1; }
cat $O/band_probe.json
timeout -k 10 200 python3 scripts/upload_probe.py 40 > $O/upload_probe.json 2> $O/upload_probe.err || { tail -20 $O/upload_probe.err; exit 1; }
cat $O/upload_probe.json
for EX in allgather owner; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo --shared-device --exchange $EX --no-cpu-baseline --no-upload --band-steps 5 > $O/rehearsal_$EX.json 2> $O/rehearsal_$EX.err
  rc=$?; echo "rehearsal $EX rc $rc"; tail -c 400 $O/rehearsal_$EX.json; [ $rc -eq 0 ] || { tail -30 $O/rehearsal_$EX.err; }
done
WL=4k_p8 TAG=r04i/r04_4k_p8 bash scripts/gpu_profile.sh > $O/prof_4k_p8.log 2>&1 || { tail -20 $O/prof_4k_p8.log; exit 1; }
tail -2 $O/prof_4k_p8.log
