# round 4: rehearsal of the N > 1 bench paths with 2 ranks on the one GPU (gloo), then the
# 4K p8 profile of this round's kernels (bench, kernel trace, PMC passes)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04h; mkdir -p $O
export TMPDIR=/tmp
for EX in allgather owner; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo --shared-device --exchange $EX --no-cpu-baseline --no-upload --band-steps 5 > $O/rehearsal_$EX.json 2> $O/rehearsal_$EX.err
  rc=$?; echo "rehearsal $EX rc $rc"; tail -c 600 $O/rehearsal_$EX.json; [ $rc -eq 0 ] || { tail -30 $O/rehearsal_$EX.err; }
done
WL=4k_p8 TAG=r04h/r04_4k_p8 bash scripts/gpu_profile.sh > $O/prof_4k_p8.log 2>&1 || { tail -20 $O/prof_4k_p8.log; exit 1; }
tail -2 $O/prof_4k_p8.log
