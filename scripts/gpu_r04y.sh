# the pipelined-upload leg: which prelude slows it (scripts/pipe_probe.py), twice each, fresh processes
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04y; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2; do for m in none timing batch both; do
  timeout -k 10 120 python3 scripts/pipe_probe.py $m >> $O/pipe_probe.jsonl 2>> $O/pipe_probe.err || { tail $O/pipe_probe.err; exit 1; }
done; done
cat $O/pipe_probe.jsonl
