"""bench.py — open-loop ME throughput on MI355X (BASELINE.json metric).

One step = one picture-level ME job (svtme_submit_picture_device): every 64x64
superblock (SB) of a 3840x2160 8-bit picture searched against 4 references
(L0: distance 1, 2; L1: distance 1, 2) with the preset-8 controls
(BASELINE.json configs[2], the headline "4K preset-8" configuration). The
references' and the current picture's padded pyramids are resident in HBM
before the timed region (the PA stage builds them once per picture).

--gpus N (launched with torch.distributed.run): one process per GPU; every rank
runs its own picture job (weak scaling: per-GPU work fixed) and the per-SB
records of all ranks are then all-gathered over RCCL (the picture-level exchange
the encoder's cross-SB consumers need, me_process.c:274-288). value = SBs of
all ranks / max-over-ranks time.

Also reported: the dominant kernel's roofline (k_me_sb: SURVEY.md 8(d)
algorithmic bytes per SB x SBs per launch / HIP-event kernel time on the
library's stream), and the reference's own AVX2 ME (oracle/_ref, compiled from
the reference sources) timed on this host's cores on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "svt-av1-mirror_amd"))

METRIC = "open-loop ME 64x64 superblocks/sec + achieved HBM GB/s, 4K preset-8"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

# bytes/SB = src 2688 + R x (ref windows + 680 output), nominal windows
WINDOW_BYTES = {"p8": 16798, "p6": 38121, "p8_sa64": 28241}
# the same bytes split over the three stage kernels (p8 stage breakdown of SURVEY.md 8(d):
# zz 2048 + pre-HME 2645 + 1034 + HME-L0 1081 | HME-L1 5304 | full-pel 4686 + 680 out;
# source 64x32 + 16x8 in stage A, 32x16 in stage B)
# (stage D only reads stage A's 448-B result block per SB: no window bytes)
STAGE_BYTES = {"p8": ((2176, 6808), (0, 0), (512, 5304), (0, 4686 + 680))}
STAGE_NAMES = ("k_stage_a", "k_stage_d", "k_stage_b", "k_stage_c1+k_stage_e")

WORKLOADS = {
    "4k_p8": dict(w=3840, h=2160, mode=8, tl=1, l0=(7, 6), l1=(9, 10), windows="p8", ten_bit=False,
                  desc="3840x2160 8-bit preset 8, 4 refs (L0 d=1,2; L1 d=1,2), open-loop ME"),
    "1080p_p8": dict(w=1920, h=1080, mode=8, tl=1, l0=(7,), l1=(), windows="p8_sa64", ten_bit=False, sa64=True,
                     desc="1920x1080 8-bit preset 8, 1 ref (L0 d=1), ME area override 64x64 "
                          "(8x8-variance resize and sr-adjust off: 4096 positions/SB), open-loop ME"),
    "4k10_p6": dict(w=3840, h=2160, mode=6, tl=1, l0=(7,), l1=(9,), windows="p6", ten_bit=True,
                    desc="3840x2160 10-bit preset 6 (8-bit MSB search), 2 refs, open-loop ME"),
    "8k_p8": dict(w=7680, h=4320, mode=8, tl=1, l0=(7, 6), l1=(9, 10), windows="p8", ten_bit=False,
                  desc="7680x4320 8-bit preset 8, 4 refs, open-loop ME"),
}


def bytes_per_sb(windows: str, refs: int) -> int:
    return 2688 + refs * (WINDOW_BYTES[windows] + 680)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="4k_p8", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-seconds of the baseline sample")
    ap.add_argument("--kernel-samples", type=int, default=10)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl")
    else:
        torch.cuda.set_device(local_rank)

    import svtme as S

    wl = WORKLOADS[args.workload]
    W, H = wl["w"], wl["h"]
    syn = S.Synth(W, H)
    ts = sorted(set((8,) + tuple(wl["l0"]) + tuple(wl["l1"])))
    frames = {t: (syn.frame10(t) if wl["ten_bit"] else syn.frame(t)) for t in ts}

    gpu = S.GpuME(local_rank)
    base = 100 * rank  # each rank owns its own picture (weak scaling)
    for t, f in frames.items():
        gpu.upload(base + t, f)
    res = S.input_resolution_of(W, H)
    ctrl = S.derive_controls(wl["mode"], 35, res, wl["tl"])
    if wl.get("sa64"):  # fixed 64x64 full-pel area
        ctrl.me_sa.sa_min.width = ctrl.me_sa.sa_min.height = 64
        ctrl.me_sa.sa_max.width = ctrl.me_sa.sa_max.height = 64
        ctrl.me_8x8_var_enabled = 0
        ctrl.enable_me_sr_adjustment = 0
    job = S.make_job(W, H, ctrl, base + 8, [base + t for t in wl["l0"]], [base + t for t in wl["l1"]],
                     temporal_layer_index=wl["tl"], enable_me_8x8=(res <= S.RES_720P), ref_count_used=(3, 2))
    R = S.ref_slots(job)
    n_sb = S.sb_total(job.width, job.height)
    rec_bytes = n_sb * R * S.REF_RECORD_DTYPE.itemsize
    sb_bytes = n_sb * S.SB_RESULT_DTYPE.itemsize
    dev = torch.device("cuda", local_rank)
    d_rec = torch.empty(rec_bytes, dtype=torch.uint8, device=dev)
    d_sb = torch.empty(sb_bytes, dtype=torch.uint8, device=dev)
    gathered = torch.empty(rec_bytes * world, dtype=torch.uint8, device=dev) if world > 1 else None
    ext = torch.cuda.ExternalStream(gpu.stream(), device=dev)

    def step():
        gpu.submit_device(job, d_rec.data_ptr(), d_sb.data_ptr())
        if world > 1:
            with torch.cuda.stream(ext):
                dist.all_gather_into_tensor(gathered, d_rec)

    for _ in range(args.warmup):
        step()
    gpu.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    gpu.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ms_per_step = elapsed / args.steps * 1e3
    value = n_sb * world * args.steps / elapsed

    # dominant kernel: k_me_sb timed with HIP events on the library's stream
    gpu.set_timing(True)
    kms, sms = [], []
    for _ in range(args.kernel_samples):
        gpu.submit_device(job, d_rec.data_ptr(), d_sb.data_ptr())
        kms.append(gpu.kernel_ms())
        sms.append([gpu.stage_ms(i) for i in range(len(STAGE_NAMES))])
    gpu.set_timing(False)
    k_avg_ms = float(np.mean(kms))
    s_avg_ms = np.mean(np.array(sms), axis=0)
    bps = bytes_per_sb(wl["windows"], R)
    achieved = bps * n_sb / (k_avg_ms * 1e-3) / 1e9
    stages = {}
    for i, name in enumerate(STAGE_NAMES):
        if s_avg_ms[i] <= 0:  # concurrent SB-band parts: no per-stage split
            continue
        st = {"avg_ms": round(float(s_avg_ms[i]), 4)}
        if wl["windows"] in STAGE_BYTES:
            src_b, per_ref = STAGE_BYTES[wl["windows"]][i]
            b = (src_b + R * per_ref) * n_sb
            if b:
                st["bytes_per_launch"] = b
                st["achieved_gbps"] = round(b / (float(s_avg_ms[i]) * 1e-3) / 1e9, 1)
        stages[name] = st
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_{args.workload}.json")
    if os.path.exists(pmc_path):
        with open(pmc_path) as fh:
            traffic = json.load(fh).get("hbm_bytes_per_launch")

    # parity of this run's records against the CPU checker (same picture)
    recs = np.frombuffer(d_rec.cpu().numpy().tobytes(), dtype=S.REF_RECORD_DTYPE).reshape(n_sb, R)
    cpu_baseline = None
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu_baseline, parity = cpu_leg(S, wl, job, frames, recs, args.cpu_seconds)

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "SB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (integer PCG32 panning texture, SURVEY.md 8(d)); pyramids resident in HBM",
            "config": {"workload": wl["desc"], "sbs_per_picture": n_sb, "refs": R,
                       "parallelism": f"one picture job per GPU x {world}, RCCL all-gather of SB records"},
            "sb_ref_per_s": round(value * R, 1),
            "algorithmic_hbm_gbps": round(bps * value / 1e9, 1),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                         "kernel": "ME pass = k_stage_a + k_stage_d + k_stage_b + k_stage_c1 + k_stage_e (one picture job)",
                         "kernel_avg_ms": round(k_avg_ms, 4), "bytes_per_launch": bps * n_sb,
                         "stages": stages},
            "cpu_baseline": cpu_baseline,
            "parity_vs_cpu": parity,
        }
        print(json.dumps(out), flush=True)
    gpu.close()
    if world > 1:
        dist.destroy_process_group()


def cpu_leg(S, wl, job, frames, gpu_recs, cpu_seconds):
    """The reference's own ME (motion_estimation.c + its AVX2 kernels, compiled
    from source into oracle/_ref) on this host, AVX2 capped as --asm avx2."""
    kind = "reference"
    try:
        S.load_ref().svtref_set_simd(1)
        checker = "ref"
    except Exception:
        kind, checker = "port", "oracle"
    threads = min(16, os.cpu_count() or 1)
    pyr = {t: S.build_host_pyramid(f, "oracle") for t, f in frames.items()}
    refs = {}
    for i, t in enumerate(wl["l0"]):
        refs[(0, i)] = pyr[t]
    for i, t in enumerate(wl["l1"]):
        refs[(1, i)] = pyr[t]
    cjob = S.make_job(wl["w"], wl["h"], job.ctrl, 8, wl["l0"], wl["l1"], temporal_layer_index=wl["tl"],
                      enable_me_8x8=bool(job.enable_me_8x8), ref_count_used=(3, 2))
    n_sb = S.sb_total(cjob.width, cjob.height)
    # first pass: parity + calibration
    t0 = time.perf_counter()
    recs, _ = S.run_checker(cjob, pyr[8], refs, checker, nthreads=threads, with_sb_results=False)
    first = time.perf_counter() - t0
    parity = not S.compare_records(recs, gpu_recs)
    # bounded sample: repeat whole-picture passes up to ~cpu_seconds of CPU time
    reps = max(1, int(cpu_seconds / max(first * threads, 1e-3)))
    t0 = time.perf_counter()
    for _ in range(reps):
        S.run_checker(cjob, pyr[8], refs, checker, nthreads=threads, with_sb_results=False)
    el = time.perf_counter() - t0
    cpu_model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return ({"value": round(n_sb * reps / el, 1), "unit": "SB/s", "cores": threads, "kind": kind,
             "sample": f"{reps} pass(es) over the full picture ({n_sb} SBs x {S.ref_slots(cjob)} refs), "
                       f"{threads} threads, {'reference AVX2 kernels' if kind == 'reference' else 'C restatement'}, "
                       f"{el:.2f} s wall, CPU: {cpu_model}"}, parity)


if __name__ == "__main__":
    main()
