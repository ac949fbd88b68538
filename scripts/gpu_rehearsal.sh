# The N > 1 path of bench.py rehearsed on a one-GPU box: 2 ranks (torch.distributed.run,
# one process each) on HIP device 0 with gloo standing in for RCCL -- every multi-rank
# code path (rank self-check, chunked search, record exchange both ways, the band_8k
# split with the three input distributions) runs through the GPU kernels; the
# collective timings are gloo's, not xGMI's.
# usage: [NPROC=2] bash scripts/gpu_rehearsal.sh
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/rehearsal; mkdir -p $O
for EX in owner allgather; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node ${NPROC:-2} --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus ${NPROC:-2} --steps 5 --warmup 2 --backend gloo --shared-device --exchange $EX \
    --no-cpu-baseline --no-upload --band-steps 5 > $O/rehearsal_$EX.json 2> $O/rehearsal_$EX.err \
    || { echo "rehearsal $EX failed"; tail -30 $O/rehearsal_$EX.err; exit 1; }
  tail -1 $O/rehearsal_$EX.json | python3 -c "import json,sys; d=json.load(sys.stdin); b=d['band_8k']; print('$EX', d['ranks'], d['config']['parallelism'], b['distribute_ms'], b['step_ms'])"
done
