cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/psweep
for r in 1 2; do for P in 4 8 16; do
timeout -k 10 200 python3 bench.py --pictures $P --steps 20 --warmup 5 --no-cpu-baseline --band-steps 0 --no-upload > gpurun_out/psweep/p${P}_r$r.json 2>gpurun_out/psweep/p${P}_r$r.err || { tail gpurun_out/psweep/p${P}_r$r.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['stages'])" gpurun_out/psweep/p${P}_r$r.json
done; done
