# round 4: the N > 1 path rehearsed on the one GPU (2 ranks, gloo, shared device) with the current
# bench (band_8k on two lanes per rank), both exchanges
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04v; mkdir -p $O; export TMPDIR=/tmp
for EX in owner allgather; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo --shared-device --exchange $EX --no-cpu-baseline --no-upload --band-steps 5 > $O/rehearsal_$EX.json 2> $O/rehearsal_$EX.err
  rc=$?; echo "rehearsal $EX rc $rc"; tail -c 600 $O/rehearsal_$EX.json; [ $rc -eq 0 ] || { tail -30 $O/rehearsal_$EX.err; exit 1; }
done
