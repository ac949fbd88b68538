# round 4: HIP API trace of the first-job probe (what the first TF-ME submission waits for)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04s; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --stats -d "$GRAFT_REPO_ROOT/$O/trace" -o run --output-format csv -- python3 scripts/first_job_probe.py > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
tail -2 $O/probe.log
