"""bench.py — open-loop ME throughput on MI355X (BASELINE.json metric).

Workload (default): BASELINE.json configs[2], the metric's "4K preset-8": every
64x64 superblock (SB) of a 3840x2160 8-bit picture searched against 4
references (L0 distance 1, 2; L1 distance 1, 2) with the preset-8 controls of
svt_aom_sig_deriv_me. Pyramids of the pictures and their references are
resident in HBM before the timed region (the PA stage builds them once per
picture). --workload picks another BASELINE config (svt-av1-mirror_amd/workloads.py).
A step writes the whole output of svt_aom_motion_estimation_b64 for every SB
(motion_estimation.c:3076-3153): the per-reference records (best MV + SAD of
the 85 PUs, HME / zz state) AND the per-SB results (candidate arrays,
me_distortion, distortions, GM flags: svtme_sb_result, :2520-3007), which is
what cpu_baseline times. The steps' pictures are consecutive pictures of one
sequence (each the current picture once, the reference of its neighbours),
all resident; consecutive steps take the next pictures (24 sets, --job-sets),
so every step publishes a new job table and the pyramids the steps read
(1.1 GB at 4K) are far beyond the 256 MiB Infinity Cache.

One step, on N GPUs (one process per GPU, torch.distributed over RCCL): 4 N
pictures (the encoder keeps several look-ahead pictures' ME in flight; the
north star's C host batches whole pictures), each split into N equal SB
chunks (SBs are independent given the picture controls); rank
r searches chunk r of every picture in ONE launch (svtme_submit_batch_device),
then each picture's chunks go to the rank that owns it (rank j owns pictures
4j..4j+3: the process whose picture-level consumers read every SB of them) in
one all_to_all_single per step over RCCL (device buffers, on a communication
stream overlapped with the next step's ME): 4 (N-1)/N pictures' records and
per-SB results per rank per step. --exchange allgather gives every rank every picture instead
(SURVEY.md 8(e)'s all_gather_into_tensor; N x the bytes per rank, the 8K
single-picture band split's exchange, and the fallback when the pictures of
a step do not divide over the ranks). Per-GPU work is four pictures' worth of
SBs at every N: "scaling" is weak. value = SBs of all pictures / max-over-ranks
wall time. "overlapped" reports one picture per GPU per step with consecutive
steps alternating the library's two submission lanes (own streams and
scratch: one step's workgroups fill the CUs while the previous one drains, as
the reference's ME threads work on several pictures at once); its kernels
overlap, so it is a chip-level rate beside the per-kernel roofline.

roofline: the ME pass (the five stage kernels, back to back on the library's
stream) — algorithmic bytes per pass (bytes/SB x SBs per
launch) / the pass's average device time, from two HIP events recorded on
that stream around the timed region. Every stage kernel is listed with its
own duration (start/stop events attached to its dispatch packets,
hipExtLaunchKernelGGL, over --kernel-samples further steps; the rocprofv3
kernel trace under profiles/ agrees) and, at p8, its own byte share;
`traffic` = HBM bytes per pass from this round's rocprofv3 FETCH_SIZE (x2,
gfx950) + WRITE_SIZE passes, committed under profiles/ (scripts/gpu_profile.sh).

cpu_baseline: the reference's own ME (motion_estimation.c + its AVX2 kernels,
compiled from the reference sources into oracle/_ref) on this host's cores
(every CPU this process may use: affinity and cgroup quota), on a bounded
sample of whole-picture passes of the same job, rank 0 at N = 1 only.
"""
import argparse
import ctypes as C
import glob
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "svt-av1-mirror_amd"))

METRIC = "open-loop ME 64x64 superblocks/sec + achieved HBM GB/s, 4K preset-8"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md, chip-level parameters)
# SAD-instruction roof measured on MI355X (scripts/ubench_sad.hip, profiles/r02_ubench_sad.json): v_sad_u8
# 150.3 T absdiff/s (0.96 wave-instr/clk/CU), v_qsad_pk_u16_u8 142.6 T/s (17.6 clk per wave-instr per SIMD)
SAD_PEAK_T = 150.3
STAGES = ("k_stage_a", "k_stage_d", "k_stage_b", "k_stage_c1", "k_stage_e")
STAGES_FUSED = ("k_hme", "-", "-", "k_stage_c1", "k_stage_e")  # k_hme = stages A + D + B (+ C1 + E) in one launch
# SURVEY.md 8(d) p8 byte split over the stage kernels: zz 2048 + pre-HME 2645 + 1034 +
# HME-L0 1081 (+ source 64x32 + 16x8) | HME-L1 5304 (+ source 32x16) | full-pel 4686 + 680 out
STAGE_BYTES_P8 = {"k_stage_a": (2176, 6808), "k_stage_d": (0, 0), "k_stage_b": (512, 5304),
                  "k_stage_c1": (0, 4686), "k_stage_e": (0, 680), "k_hme": (2688, 12112)}
# the whole pass in k_hme (fused full-pel + decode): every byte of the pass
STAGE_BYTES_P8_ALL = (2688, 16798 + 680)
PICTURES_PER_GPU = 4  # pictures of one step per GPU, one batched launch (--pictures overrides)
MAX_BATCH = 16  # SVTME_MAX_BATCH_JOBS (include/svtme.h): jobs of one batched launch


def host_cores():
    """CPUs this process may run on: affinity, capped by the cgroup CPU quota."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, p = fh.read().split()[:2]
        if q != "max":
            n = min(n, max(1, math.ceil(int(q) / int(p))))
    except (OSError, ValueError):
        pass
    return n


def kernel_code_sha():
    """sha256 of the device sources of the ME pass (stage kernels + shared headers)."""
    import hashlib

    h = hashlib.sha256()
    for f in ("svtme_stages.hip", "svtme_me_common.h", "svtme_device.h"):
        with open(os.path.join(ROOT, "svt-av1-mirror_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def latest_profile(workload):
    """pmc_summary.json under profiles/*_<workload>/ taken on THIS build's stage
    kernels (same code_sha), or (None, None)."""
    sha = kernel_code_sha()
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{workload}", "pmc_summary.json"))):
        with open(path) as fh:
            prof = json.load(fh)
        if prof.get("code_sha") == sha:
            return prof, os.path.relpath(path, ROOT)
    return None, None


def main():
    import workloads as W

    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5,
                    help="untimed steps first (the defaults are the driver's window; the GPU's clocks ramp over the "
                         "first ~25 ms of load, so this window runs ~10 %% below the steady state that "
                         "`steady_state` reports, DESIGN.md 4)")
    ap.add_argument("--steady-steps", type=int, default=200,
                    help="steps of the secondary steady-state measurement (after 300 more untimed steps, once the "
                         "clocks have ramped); 0 skips it")
    ap.add_argument("--workload", default="4k_p8", choices=sorted(W.WORKLOADS))
    ap.add_argument("--pictures", type=int, default=0,
                    help=f"pictures per step (default: {PICTURES_PER_GPU} per GPU; several go in one batched launch)")
    ap.add_argument("--kernel-samples", type=int, default=20, help="steps timed per kernel after the timed region")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-single-picture", "--no-alt-mode", dest="no_alt", action="store_true",
                    help="skip the timing of the other picture count (batched / single picture)")
    ap.add_argument("--no-upload", action="store_true", help="skip the host-upload (PCIe-inclusive) timing")
    ap.add_argument("--no-records-only", action="store_true",
                    help="skip the secondary timing of the same steps writing the records alone (no per-SB results)")
    ap.add_argument("--records-only", action="store_true",
                    help="the timed steps write the records alone (default: records + per-SB results, the whole "
                         "output of svt_aom_motion_estimation_b64)")
    ap.add_argument("--job-sets", type=int, default=0,
                    help="job sets the steps rotate over: consecutive pictures of one sequence, each resident "
                         "once (default 24: more than the 16 job tables the library keeps, so every step "
                         "publishes its table)")
    ap.add_argument("--lanes", type=int, default=2, choices=(1, 2),
                    help="submission lanes the timed steps alternate over (svtme_submit_batch_device_lane); the "
                         "overlapped two-lane rate is reported beside the one-lane value")
    ap.add_argument("--launch-pictures", type=int, default=0,
                    help="pictures per launch (default: all of a step's pictures, at most 16); with two lanes "
                         "consecutive launches alternate lanes, so one launch's tail overlaps the next")
    ap.add_argument("--exchange", default="owner", choices=("owner", "allgather"),
                    help="N > 1 record exchange: each picture's chunks to its owner rank (all_to_all_single), or "
                         "every picture to every rank (all_gather_into_tensor)")
    ap.add_argument("--cpu-seconds", type=float, default=30.0, help="target CPU-seconds of the baseline sample")
    ap.add_argument("--band-steps", type=int, default=30,
                    help="steps of the band_8k sub-measurement (one 8K p8 picture split over the N GPUs, SURVEY.md "
                         "8(e)); 0 skips it")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI; gloo: a rehearsal of the "
                         "multi-rank code paths, e.g. several ranks on one GPU with --shared-device)")
    ap.add_argument("--shared-device", action="store_true",
                    help="every rank on HIP device 0 (rehearsal of the N > 1 path on a one-GPU box, with gloo)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = 0 if args.shared_device else int(os.environ.get("LOCAL_RANK", "0"))

    import torch

    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist

        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group("gloo")
        # self-check of the launch: the process group spans exactly the ranks the launcher started
        if dist.get_world_size() != world or dist.get_rank() != rank:
            raise SystemExit(f"torch.distributed has rank {dist.get_rank()} of {dist.get_world_size()}, the launcher "
                             f"set RANK={rank} WORLD_SIZE={world}")
        if args.gpus != world:
            raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    import svtme as S
    import svtme_dist as D

    name = args.workload
    wl = W.WORKLOADS[name]
    Wd, Ht = wl["w"], wl["h"]
    P = args.pictures or PICTURES_PER_GPU * world
    P_alt = world  # one picture per GPU per step: the "overlapped" mode reported beside the main one
    n_sb = S.sb_total(Wd, Ht)
    slots = D.chunk_slots(n_sb, world)
    begin, count = D.sb_chunk(n_sb, rank, world)

    gpu = S.GpuME(local_rank)
    syn = S.Synth(Wd, Ht)
    offs = sorted(set((0,) + tuple(t - 8 for t in wl["l0"]) + tuple(t - 8 for t in wl["l1"])))
    PM = max(P, P_alt)
    # The pictures of the steps form one sequence, as an encoder's do: picture i (of NS x PM) is
    # frame 8 + i searched against frames 8 + i -+ 1, 2 (picture numbers = content times, so the
    # reference distances, and with them the search areas, are the workload's); consecutive
    # pictures share references, every picture is resident once. Step k submits set k % NS, the
    # pictures [PM (k % NS), PM (k % NS + 1)): with NS > 16 (the library's job-table ring) every
    # step publishes a new job table, and the sequence's pyramids (1.1 GB at 4K) are far beyond
    # the 256 MiB Infinity Cache. Picture 0 is the workload's own job (base 0), the one the CPU
    # baseline checks.
    NS = args.job_sets or 24
    lo_t = 8 + min(offs)
    hi_t = 8 + NS * PM - 1 + max(offs)
    for t in range(lo_t, hi_t + 1):
        gpu.upload(t, W.workload_frame(name, syn, t))
    sets = [[W.workload_job(name, base=si * PM + p, sb_begin=begin, sb_count=count) for p in range(PM)]
            for si in range(NS)]
    jobs = sets[0]
    R = S.ref_slots(jobs[0])
    rec = S.REF_RECORD_DTYPE.itemsize
    sbsz = S.SB_RESULT_DTYPE.itemsize
    with_sb = jobs[0].me_type != S.ME_MCTF and not args.records_only  # TF-ME jobs have no per-SB results
    # one picture's chunk: its records, then (PA-ME) its per-SB results; both go to the owner rank
    rec_bytes = slots * R * rec
    chunk_bytes = rec_bytes + (slots * sbsz if with_sb else 0)
    chunk_bytes = (chunk_bytes + 255) & ~255
    dev = torch.device("cuda", local_rank)
    local = [torch.zeros(PM * chunk_bytes, dtype=torch.uint8, device=dev) for _ in range(2)]
    # the owner exchange needs each step's pictures to divide over the ranks
    owner = world > 1 and args.exchange == "owner" and P % world == 0 and P_alt % world == 0
    exchange = None if world == 1 else ("owner (all_to_all_single)" if owner else "allgather (all_gather_into_tensor)")
    gathered = [torch.empty((1 if owner else world) * PM * chunk_bytes, dtype=torch.uint8, device=dev)
                for _ in range(2)] if world > 1 else None
    NL = args.lanes
    exts = [torch.cuda.ExternalStream(gpu.lane_stream(l), device=dev) for l in range(max(2, NL))]
    ext = exts[0]
    comm = torch.cuda.Stream(device=dev) if world > 1 else None
    me_done = [torch.cuda.Event() for _ in range(2)]
    g_done = [torch.cuda.Event() for _ in range(2)]
    used = [False, False]

    LP = min(args.launch_pictures or MAX_BATCH, MAX_BATCH)
    nlaunch = [0]

    def step(i, n_pic=P, nl=NL, lp=LP, sb=None):
        b = i & 1
        sb = with_sb if sb is None else sb
        js = sets[i % NS]
        if used[b] and world > 1:
            for l in range(nl):
                exts[l].wait_event(g_done[b])  # the gather of step i-2 has read local[b]
        lanes_used = set()
        base = local[b].data_ptr()
        for g0 in range(0, n_pic, lp):  # at most SVTME_MAX_BATCH_JOBS jobs per launch
            g1 = min(n_pic, g0 + lp)
            lane = nlaunch[0] % nl  # two lanes: consecutive launches alternate, their kernels overlap on the GPU
            nlaunch[0] += 1
            lanes_used.add(lane)
            gpu.submit_batch_device(js[g0:g1], [base + p * chunk_bytes for p in range(g0, g1)],
                                    [base + p * chunk_bytes + rec_bytes for p in range(g0, g1)] if sb else None,
                                    lane=lane)
        if world > 1:
            for l in sorted(lanes_used):
                me_done[b].record(exts[l])
                comm.wait_event(me_done[b])
            if owner:  # this step's n_pic chunks: n_pic / world pictures per owner
                D.exchange_to_owners_device(local[b][:n_pic * chunk_bytes], gathered[b][:n_pic * chunk_bytes], dist,
                                            stream=comm)
            else:
                D.gather_chunks_device(local[b], gathered[b], dist, stream=comm)
            g_done[b].record(comm)
        used[b] = True

    def fence():
        gpu.sync()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    fence()  # the buffers' zero fills (torch's stream) before the library's streams write them
    for i in range(args.warmup):
        step(i)
    fence()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    join = torch.cuda.Event()

    def end_on_lane0(ev):  # lane 0 waits for the other lanes' queues, then records ev
        for l in range(1, len(exts)):
            join.record(exts[l])
            ext.wait_event(join)
        ev.record(ext)
    t0 = time.perf_counter()
    ev0.record(ext)
    for i in range(args.steps):
        step(args.warmup + i)
    host_submit_s = time.perf_counter() - t0  # the host's share: how far ahead of the GPU it ran
    end_on_lane0(ev1)
    fence()
    elapsed = time.perf_counter() - t0
    device_ms = ev0.elapsed_time(ev1) / args.steps  # the library stream's time per step (HIP events)
    # per-kernel durations: start/stop events attached to the stage dispatches
    # themselves (hipExtLaunchKernelGGL) over a sample of further steps
    gpu.set_timing(True)
    for i in range(args.kernel_samples):  # one lane, one launch per step: kernel durations without overlap
        step(args.warmup + args.steps + i, P, 1, MAX_BATCH)
    fence()
    gpu.set_timing(False)
    n_timed, stage_ms = gpu.timing_read()
    # overlapped mode: one picture per GPU per step, consecutive steps on the two
    # submission lanes (the next step's workgroups fill the CUs while the previous
    # step drains; kernels overlap, so this is a chip-level rate, not a per-kernel one)
    alt_ms = None
    if not args.no_alt:
        for i in range(args.warmup):
            step(i, P_alt, 2, MAX_BATCH)
        fence()
        t0a = time.perf_counter()
        for i in range(args.steps):
            step(args.warmup + i, P_alt, 2, MAX_BATCH)
        fence()
        alt_ms = (time.perf_counter() - t0a) / args.steps * 1e3
        if world > 1:
            ta = torch.tensor([alt_ms], dtype=torch.float64, device=dev)
            dist.all_reduce(ta, op=dist.ReduceOp.MAX)
            alt_ms = float(ta.item())
    # secondary: the same steps writing the records alone (the north star's best MV + SAD per PU,
    # without the candidate arrays / distortions / GM flags of svtme_sb_result)
    ro_ms = None
    if with_sb and not args.no_records_only:
        for i in range(args.warmup):
            step(i, sb=False)
        fence()
        t0s = time.perf_counter()
        for i in range(args.steps):
            step(args.warmup + i, sb=False)
        fence()
        ro_ms = (time.perf_counter() - t0s) / args.steps * 1e3
        if world > 1:
            ts = torch.tensor([ro_ms], dtype=torch.float64, device=dev)
            dist.all_reduce(ts, op=dist.ReduceOp.MAX)
            ro_ms = float(ts.item())
    # secondary: the same steps in steady state (the clocks ramp over the first ~25 ms of
    # load): 300 more untimed steps, then --steady-steps timed in blocks that
    # alternate the whole output and the records alone (their ratio: the cost of the per-SB
    # results at equal clocks); never `value`
    steady = None
    if args.steady_steps > 0:
        for i in range(300):
            step(i)
        fence()
        blk = max(1, args.steady_steps // 4)
        t_sb = t_ro = 0.0
        for r in range(4):
            sb_blk = with_sb and r % 2 == 1  # records-only blocks first, the whole output second
            fence()
            t0s = time.perf_counter()
            for i in range(blk):
                step(300 + r * blk + i, sb=sb_blk)
            fence()
            dt = time.perf_counter() - t0s
            if sb_blk or not with_sb:
                t_sb += dt
            else:
                t_ro += dt
        nb = 2 if with_sb else 4
        st_ms = t_sb / (nb * blk) * 1e3
        ro_st = t_ro / (2 * blk) * 1e3 if with_sb else None
        if world > 1:
            ts = torch.tensor([st_ms, ro_st or 0.0], dtype=torch.float64, device=dev)
            dist.all_reduce(ts, op=dist.ReduceOp.MAX)
            st_ms, ro_st = float(ts[0].item()), (float(ts[1].item()) if with_sb else None)
        steady = {"ms_per_step": round(st_ms, 4), "value": round(n_sb * P / (st_ms * 1e-3), 1),
                  "untimed_steps_before": 300, "steps": nb * blk,
                  "records_only": None if ro_st is None else {
                      "ms_per_step": round(ro_st, 4), "value": round(n_sb * P / (ro_st * 1e-3), 1),
                      "sb_results_cost": round(st_ms / ro_st - 1.0, 4)},
                  "note": "the main line's steps after the GPU has been busy for ~60 ms (clocks ramped: in-kernel "
                          "clock 2.24 -> 2.38 GHz over the first 12 ms of load, profiles/r05_warmup/), in blocks "
                          "alternating the whole output and the records alone; a secondary figure, `value` is "
                          "the driver's window"}
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ms_per_step = elapsed / args.steps * 1e3
    value = n_sb * P * args.steps / elapsed

    # PCIe-inclusive rate (never `value`): one picture's upload from
    # host memory (pageable numpy, and a pinned buffer) + pyramid build, synchronous
    upload = None
    if rank == 0 and not args.no_upload:
        frame = W.workload_frame(name, syn, 8)
        fn = gpu.lib.svtme_picture_upload_10bit if wl["ten_bit"] else gpu.lib.svtme_picture_upload

        def t_up(ptr, reps=10):
            t = []
            for k in range(reps + 2):
                t0u = time.perf_counter()
                gpu._check(fn(gpu.ctx, 900000 + k, ptr, Wd, Wd, Ht), "upload")
                t.append(time.perf_counter() - t0u)
                gpu.release(900000 + k)
            return float(np.median(t[2:])) * 1e3
        pageable_ms = t_up(np.ascontiguousarray(frame).ctypes.data)
        pinned = torch.from_numpy(np.ascontiguousarray(frame)).pin_memory()
        pinned_ms = t_up(pinned.data_ptr())
        me_ms = ms_per_step / P * world
        # pipelined: each step uploads a new current picture asynchronously
        # (svtme_picture_upload_async, pinned source) and searches it against the
        # resident references on the next submission lane; 8 pictures rotate, so an
        # upload waits only for the search of the picture it replaces, 8 steps back
        # (scripts/upload_probe.py: 4 rotating pictures on one lane serialise more)
        # (each rotating picture has its own resident references at the workload's distances:
        # picture numbers set the reference distances, and so the search areas)
        NP = 8
        pbase = [910000 + 64 * k for k in range(NP)]
        pjobs = [W.workload_job(name, base=b) for b in pbase]
        for b in pbase:
            for t in offs:
                if t != 0:
                    gpu.upload(b + 8 + t, W.workload_frame(name, syn, 8 + t))
        pbuf = [torch.zeros(n_sb * R * S.REF_RECORD_DTYPE.itemsize, dtype=torch.uint8, device=dev) for _ in range(2)]

        def pipe(i):
            gpu.upload_async(pbase[i % NP] + 8, pinned.data_ptr(), Wd, Ht)
            gpu.submit_batch_device([pjobs[i % NP]], [pbuf[i & 1].data_ptr()], lane=i & 1)
        for i in range(2 * NP):
            pipe(i)
        gpu.sync()
        reps = 80
        t0p = time.perf_counter()
        for i in range(reps):
            pipe(i)
        gpu.sync()
        pipe_ms = (time.perf_counter() - t0p) / reps * 1e3
        # the same loop with the uploads only (the copy engine's rate)
        t0p = time.perf_counter()
        for i in range(reps):
            gpu.upload_async(pbase[i % NP] + 8, pinned.data_ptr(), Wd, Ht)
        gpu.sync()
        up_only_ms = (time.perf_counter() - t0p) / reps * 1e3
        for b in pbase:
            for t in offs:
                gpu.release(b + 8 + t)
        upload = {"pageable_ms_per_picture": round(pageable_ms, 4), "pinned_ms_per_picture": round(pinned_ms, 4),
                  "picture_bytes": int(frame.nbytes),
                  "pcie_inclusive_sb_per_s": round(n_sb / ((pinned_ms + me_ms) * 1e-3), 1),
                  "pipelined_ms_per_picture": round(pipe_ms, 4),
                  "pipelined_sb_per_s": round(n_sb / (pipe_ms * 1e-3), 1),
                  "async_upload_only_ms_per_picture": round(up_only_ms, 4),
                  "note": "upload + pyramid build of one picture from host memory, synchronous; pipelined: "
                          "asynchronous upload of each step's current picture (pinned) overlapped with the "
                          "searches, one picture per launch on alternating lanes, 8 pictures rotating"}

    # roofline of the ME pass on this rank (one batched launch per stage)
    sbs_launch = count * P
    bps = W.bytes_per_sb(wl["windows"], R)
    kern_ms = float(sum(stage_ms))
    bytes_launch = bps * sbs_launch
    achieved = bytes_launch / (device_ms * 1e-3) / 1e9
    stages = {}
    fused = stage_ms[0] > 0 and stage_ms[1] <= 0 and stage_ms[2] <= 0
    names = list(STAGES_FUSED if fused else STAGES)
    lib = S.load_product()
    lib.svtme_fp_wide_lds.argtypes = [C.POINTER(S.Controls)]
    lib.svtme_fp_wide_lds.restype = C.c_bool
    if lib.svtme_fp_wide_lds(C.byref(jobs[0].ctrl)):
        names[3] = "k_fp_wide"  # the wide full-pel stage with its window in LDS
    lib.svtme_l1_full.argtypes = [C.POINTER(S.Controls)]
    lib.svtme_l1_full.restype = C.c_bool
    if not fused and lib.svtme_l1_full(C.byref(jobs[0].ctrl)):
        names[2] = "k_l1_full"  # full-SAD HME-L1, two quadrants per wavefront
    lib.svtme_l0_full_job.argtypes = [C.POINTER(S.Job)]
    lib.svtme_l0_full_job.restype = C.c_bool
    if not fused and lib.svtme_l0_full_job(C.byref(jobs[0])):
        names[0] = "k_l0_full"  # full-SAD zz + HME-L0, one wavefront per (SB, slot)
    for k, st in enumerate(names):
        if stage_ms[k] <= 0:
            continue
        e = {"avg_ms": round(stage_ms[k], 4), "share": round(stage_ms[k] / kern_ms, 3)}
        if wl["windows"] == "p8":
            src_b, per_ref = STAGE_BYTES_P8_ALL if (fused and stage_ms[3] <= 0) else STAGE_BYTES_P8[st]
            sb_b = (src_b + R * per_ref) * count * min(P, MAX_BATCH)  # one kernel launch
            if sb_b:
                e["bytes_per_launch"] = sb_b
                e["achieved_gbps"] = round(sb_b / (stage_ms[k] * 1e-3) / 1e9, 1)
                e["frac"] = round(e["achieved_gbps"] / HBM_PEAK_GBPS, 4)
        stages[st] = e
    dom = max(stages, key=lambda s: stages[s]["avg_ms"]) if stages else None
    pass_gbps = achieved
    if dom and "achieved_gbps" in stages[dom]:  # the dominant kernel's own launches (one lane, HIP events)
        achieved = stages[dom]["achieved_gbps"]
    prof, prof_path = latest_profile(name)
    traffic = None
    if prof and prof.get("hbm_bytes_per_launch") and prof.get("sbs_per_launch") == sbs_launch:
        traffic = int(prof["hbm_bytes_per_launch"])
    absdiff = W.ABSDIFF_PER_SB_REF[wl["windows"]] * R * sbs_launch
    sad_rate = absdiff / (device_ms * 1e-3) / 1e12
    # measured DRAM rate of the dominant kernel: rocprofv3 HBM bytes per launch (same code) / its duration
    dram = None
    if traffic and dom:
        dram_gbps = traffic / (stages[dom]["avg_ms"] * 1e-3) / 1e9
        dram = {"gbps": round(dram_gbps, 1), "frac": round(dram_gbps / HBM_PEAK_GBPS, 4),
                "note": "measured HBM bytes per launch (traffic) / the kernel's average duration: the share of "
                        "the 8 TB/s the kernel really draws; the algorithmic frac counts every search window "
                        "as read from HBM, most of which neighbouring SBs' workgroups find in L2 / MALL"}

    # what bounds the dominant kernel, from the evidence: the measured DRAM rate and the SAD-unit rate
    dram_frac = dram["frac"] if dram else None
    sad_frac = sad_rate / SAD_PEAK_T
    if dram_frac is not None and dram_frac >= 0.5:
        bound, limiter = "hbm", "measured HBM traffic at >= half of the 8 TB/s peak"
    elif sad_frac >= 0.5:
        bound, limiter = "valu", "SAD instructions (v_qsad / v_sad) at >= half of their measured roof"
    else:
        bound = "issue"
        limiter = ("issue / latency: neither HBM (dram.frac " + (f"{dram_frac:.2f}" if dram_frac is not None else "n/a")
                   + f") nor the SAD units (valu_sad.frac {sad_frac:.2f}) are at half their roof; frac is the "
                   "SURVEY.md 8(d) algorithmic-bytes rate")
    chip_gbps = bps * count * P / (ms_per_step * 1e-3) / 1e9  # this rank's algorithmic bytes per step / step time

    band = None
    if args.band_steps > 0:
        band = band_8k_leg(gpu, S, W, D, dist, world, rank, dev, exts, comm, args.band_steps, fence)

    recs = sbres = None
    if world == 1:  # the workload's own job (set 0, picture 0), as the timed steps run it, for the parity check
        chk = torch.zeros(chunk_bytes, dtype=torch.uint8, device=dev)
        gpu.submit_batch_device([sets[0][0]], [chk.data_ptr()], [chk.data_ptr() + rec_bytes] if with_sb else None,
                                lane=0)
        gpu.sync()
        raw = chk.cpu().numpy()
        recs = np.frombuffer(raw[:n_sb * R * rec].tobytes(), dtype=S.REF_RECORD_DTYPE).reshape(n_sb, R)
        if with_sb:
            sbres = np.frombuffer(raw[rec_bytes:rec_bytes + n_sb * sbsz].tobytes(), dtype=S.SB_RESULT_DTYPE)
    cpu_baseline = parity = ref_absdiff = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu_baseline, parity, ref_absdiff = cpu_leg(S, W, name, recs, sbres, args.cpu_seconds)
    valu_sad = {"achieved_T_absdiff_s": round(sad_rate, 2), "peak": SAD_PEAK_T, "frac": round(sad_rate / SAD_PEAK_T, 4),
                "absdiff_per_sb_ref": W.ABSDIFF_PER_SB_REF[wl["windows"]],
                "note": "SURVEY.md 8(d) nominal absdiff (distance-1 windows, no early exit) per launch / pass time"}
    if "k_fp_wide" in stages and wl["windows"] in W.FULLPEL_ABSDIFF_PER_SB_REF:  # the wide full-pel stage alone
        fp_absdiff = W.FULLPEL_ABSDIFF_PER_SB_REF[wl["windows"]] * R * sbs_launch
        fp_rate = fp_absdiff / (stages["k_fp_wide"]["avg_ms"] * 1e-3) / 1e12
        valu_sad["fullpel_stage"] = {"kernel": "k_fp_wide", "absdiff_per_launch": fp_absdiff,
                                     "achieved_T_absdiff_s": round(fp_rate, 2),
                                     "frac": round(fp_rate / SAD_PEAK_T, 4),
                                     "note": "full-pel absdiff (positions x 2048) per launch / k_fp_wide time"}
    if ref_absdiff:
        per_sb = ref_absdiff / n_sb
        ref_rate = per_sb * sbs_launch / (device_ms * 1e-3) / 1e12
        valu_sad.update({"reference_absdiff_per_sb": round(per_sb), "reference_T_absdiff_s": round(ref_rate, 2),
                         "reference_frac": round(ref_rate / SAD_PEAK_T, 4),
                         "reference_note": "absdiff the reference's searches evaluate on this job (early exits "
                                           "and pruning included; counted by the CPU oracle) per launch / pass "
                                           "time; the GPU also runs the pre-HME / HME-L0 searches the reference "
                                           "may skip, in the same pass (DESIGN.md 4)"})

    devices = sorted(set(gather_devices(dist, local_rank, dev)))  # (a collective: every rank)
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "SB/s",
            "n_gpus": world,
            "ranks": {"world_size_env": world, "process_group": dist.get_world_size() if dist else 1,
                      "backend": (dist.get_backend() if dist else "none (N = 1: no collective)"),
                      "rccl_version": rccl_version(torch),
                      "devices": devices},
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "host_submit_ms_per_step": round(host_submit_s * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": ("synthetic (integer PCG32 texture, SURVEY.md 8(d); " +
                     ("per-region motion and noise" if wl.get("content") == "mixed" else "global pan") +
                     "); pyramids resident in HBM"),
            "config": {"workload": wl["desc"], "name": name, "sbs_per_picture": n_sb, "refs": R,
                       "pictures_per_step": P,
                       "job_sets": NS, "resident_pyramids": hi_t - lo_t + 1,
                       "outputs": "records + svtme_sb_result" if with_sb else "records",
                       "lanes": NL,
                       "parallelism": f"{world} GPU(s): each picture split in {world} equal SB chunks, "
                                      f"rank r searches chunk r of all {P} pictures in {-(-P // LP)} launch(es) per step" +
                                      (f", launches of {min(LP, P)} picture(s) alternating the two submission lanes"
                                       if NL > 1 else "") +
                                      (f", record exchange over {'RCCL' if dist.get_backend() == 'nccl' else dist.get_backend()}"
                                       f": {exchange}" if world > 1 else "")},
            "overlapped": None if alt_ms is None else {
                "pictures_per_step": P_alt, "lanes": 2, "ms_per_step": round(alt_ms, 4),
                "value": round(n_sb * P_alt / (alt_ms * 1e-3), 1),
                "algorithmic_hbm_gbps": round(bps * n_sb * P_alt / (alt_ms * 1e-3) / 1e9, 1),
                "note": "one picture per GPU per step, consecutive steps alternating the two submission lanes "
                        "(svtme_submit_batch_device_lane): kernels of consecutive steps overlap, wall clock"},
            "records_only": None if ro_ms is None else {
                "ms_per_step": round(ro_ms, 4), "value": round(n_sb * P / (ro_ms * 1e-3), 1),
                "sb_results_cost": round(ms_per_step / ro_ms - 1.0, 4),
                "note": "the same steps writing the records alone (no svtme_sb_result), timed after the main "
                        "window and the overlapped leg, i.e. further into the clock ramp: its ratio to `value` "
                        "overstates the per-SB results' cost (steady_state.records_only alternates blocks and is "
                        "the fair comparison; --records-only times them in the main window); `value` writes both, "
                        "the whole output of svt_aom_motion_estimation_b64 that cpu_baseline times"},
            "steady_state": steady,
            "upload": upload,
            "sb_ref_per_s": round(value * R, 1),
            "algorithmic_hbm_gbps": round(bps * value / 1e9, 1),
            "roofline": {"bound": bound, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                         "kernel": "ME pass: " + " -> ".join(n for k, n in enumerate(names) if stage_ms[k] > 0) +
                                   " (one launch each, back to back on the library stream)",
                         "achieved_from": ("bytes_per_launch of the dominant kernel / its average launch "
                                           "duration (HIP events on its dispatches, one lane)"
                                           if achieved != pass_gbps else "pass bytes / pass time"),
                         "pass_gbps": round(pass_gbps, 1),
                         "pass_ms": round(device_ms, 4), "kernel_sum_ms": round(kern_ms, 4),
                         "kernel_samples": n_timed,
                         "bytes_per_launch": bytes_launch, "sbs_per_launch": sbs_launch,
                         "dominant": dom, "stages": stages, "traffic_source": prof_path,
                         "valu_sad": valu_sad,
                         "algorithmic_frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "dram": dram,
                         "chip": {"gbps": round(chip_gbps, 1), "frac": round(chip_gbps / HBM_PEAK_GBPS, 4),
                                  "note": "algorithmic bytes of one step / ms_per_step: the chip-level rate of the "
                                          "timed steps, whose launches overlap on the two lanes (frac above is one "
                                          "lane's launch alone, a lower bound on chip use)"},
                         "limiter": limiter},
            "band_8k": band,
            "cpu_baseline": cpu_baseline,
            "parity_vs_cpu": parity,
        }
        print(json.dumps(out), flush=True)
    gpu.close()
    if world > 1:
        dist.destroy_process_group()


def rccl_version(torch):
    """The RCCL (torch.cuda.nccl) version this torch build links, as a string."""
    try:
        v = torch.cuda.nccl.version()
        return ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception as e:  # noqa: BLE001 (reported, not fatal)
        return f"unavailable ({type(e).__name__})"


def gather_devices(dist, local_rank, dev):
    """The HIP device of every rank (one process per GPU: N distinct devices)."""
    if dist is None:
        return [local_rank]
    import torch

    t = torch.tensor([local_rank], dtype=torch.int64, device=dev if dist.get_backend() == "nccl" else "cpu")
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [int(o.item()) for o in out]


def band_8k_leg(gpu, S, W, D, dist, world, rank, dev, exts, comm, steps, fence):
    """SURVEY.md 8(e) / BASELINE configs[4]: ONE 7680x4320 p8 picture per step,
    its SBs split in N equal chunks (D.BandSplit): the picture's 8-bit luma plane
    reaches every rank (rank 0 uploads it from pinned host memory and an RCCL
    broadcast over xGMI fans it out, or every rank uploads its own copy over its
    PCIe link), every rank builds the pyramid on device
    (svtme_picture_upload_device_async), searches its chunk in one launch, and
    one all_gather_into_tensor over RCCL gives every rank the picture's records.
    The references (the previous pictures) stay resident, as in an encode, where
    each picture is distributed once on arrival. Timed separately: the
    distribution both ways, the search alone, the all-gather alone, and the
    pipelined step (distribution of picture i + 1 on the copy / upload streams
    while picture i is searched and gathered; consecutive pictures' searches on
    the two submission lanes, each with its own chunk buffer, so that at N = 8,
    where a rank's chunk is 1 020 workgroups against 2 048 resident slots, the
    next picture's search fills the CUs the previous one leaves); strong
    scaling: SBs of the picture / the pipelined step time."""
    import torch

    name = "8k_p8"
    wl = W.WORKLOADS[name]
    Wd, Ht = wl["w"], wl["h"]
    # two sets of resident references (the previous pictures); the current picture of step i is
    # set i & 1's picture 8, so distributing the next one waits only for the search two steps
    # back, and every job keeps the workload's reference distances
    bases = [800000, 800064]
    frames = W.workload_frames(name)
    for b in bases:
        for t, f in frames.items():  # every rank holds the full pyramids (pre-HME reaches ~1400 rows)
            if t != 8:
                gpu.upload(b + t, f)
    n_sb = S.sb_total(Wd, Ht)
    R = len(wl["l0"]) + len(wl["l1"])
    split = D.BandSplit(n_sb, R, S.REF_RECORD_DTYPE.itemsize, world, rank)
    cur = [b + 8 for b in bases]
    jobs = [W.workload_job(name, base=b, sb_begin=split.begin, sb_count=split.count) for b in bases]
    local = [torch.zeros(split.chunk_bytes, dtype=torch.uint8, device=dev) for _ in range(2)]
    out = [torch.empty(world * split.chunk_bytes, dtype=torch.uint8, device=dev) if world > 1 else None
           for _ in range(2)]
    searched, gathered = [torch.cuda.Event() for _ in range(2)], [torch.cuda.Event() for _ in range(2)]
    host = torch.from_numpy(frames[8].reshape(-1)).pin_memory() if rank == 0 or world == 1 else None
    host_all = torch.from_numpy(frames[8].reshape(-1)).pin_memory()  # the per-rank PCIe variant
    ps = D.PlaneSlices(Wd, Ht, world, rank)  # the sliced variant: this rank's rows only
    host_mine = torch.from_numpy(ps.host_rows(frames[8]).copy()).pin_memory()
    slices = [torch.zeros(ps.slice_bytes, dtype=torch.uint8, device=dev) for _ in range(2)]
    planes = [torch.empty(max(Wd * Ht, ps.plane_bytes), dtype=torch.uint8, device=dev) for _ in range(2)]
    ustream = torch.cuda.ExternalStream(gpu.upload_stream(), device=dev)
    copy = torch.cuda.Stream(device=dev)
    arrived, built = [torch.cuda.Event() for _ in range(2)], [torch.cuda.Event() for _ in range(2)]
    for b in range(2):
        built[b].record(ustream)

    def distribute(i, mode):
        b = i & 1
        copy.wait_event(built[b])  # the pyramid build two pictures back has read planes[b]
        if mode == "pcie" or world == 1:
            with torch.cuda.stream(copy):
                planes[b][: Wd * Ht].copy_(host_all, non_blocking=True)
            arrived[b].record(copy)
        elif mode == "sliced":  # every rank uploads its H/N rows, one RCCL all-gather over xGMI assembles the plane
            with torch.cuda.stream(copy):
                slices[b][: host_mine.numel()].copy_(host_mine, non_blocking=True)
            arrived[b].record(copy)
            comm.wait_event(arrived[b])
            ps.gather(slices[b], planes[b][: ps.plane_bytes], dist, stream=comm)
            arrived[b].record(comm)
        else:  # rank 0 uploads, one RCCL broadcast over xGMI fans the plane out
            if rank == 0:
                with torch.cuda.stream(copy):
                    planes[b].copy_(host, non_blocking=True)
            arrived[b].record(copy)
            comm.wait_event(arrived[b])
            D.broadcast_plane(planes[b][: Wd * Ht], dist, src=0, stream=comm)
            arrived[b].record(comm)
        ustream.wait_event(arrived[b])
        gpu.upload_device_async(cur[b], planes[b].data_ptr(), Wd, Wd, Ht)
        built[b].record(ustream)

    def search(i=0):
        b = i & 1
        gpu.submit_batch_device([jobs[b]], [local[b].data_ptr()], lane=b)

    def gather(i=0):
        b = i & 1
        searched[b].record(exts[b])
        comm.wait_event(searched[b])
        split.exchange(local[b], out[b], dist, stream=comm)
        gathered[b].record(comm)
        exts[b].wait_event(gathered[b])  # the lane's next search rewrites the chunk the gather reads

    def timed(fn):
        fence()
        t0 = time.perf_counter()
        for i in range(steps):
            fn(i)
        fence()
        ms = (time.perf_counter() - t0) / steps * 1e3
        if world > 1:
            t = torch.tensor([ms], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            ms = float(t.item())
        return ms

    modes = ("pcie",) if world == 1 else ("sliced", "broadcast", "pcie")
    for i in range(4):
        distribute(i, modes[0])
        search(i)
        if world > 1:
            gather(i)
    dist_ms = {m: timed(lambda i, m=m: distribute(i, m)) for m in modes}
    best = min(dist_ms, key=dist_ms.get)
    search_ms = timed(search)
    gather_ms = timed(lambda i: split.exchange(local[i & 1], out[i & 1], dist, stream=comm)) if world > 1 else 0.0

    def step(i):
        distribute(i, best)
        search(i)
        if world > 1:
            gather(i)
    pair_ms = timed(lambda i: (search(i), gather(i))) if world > 1 else search_ms
    step_ms = timed(step)
    for b in bases:
        for t in frames:
            gpu.release(b + t)
    return {"workload": wl["desc"] + ", one picture per step split over the GPUs", "sbs_per_picture": n_sb,
            "sbs_per_rank": split.slots, "refs": R, "steps": steps, "picture_bytes": Wd * Ht,
            "distribute_ms": {m: round(v, 4) for m, v in dist_ms.items()}, "distribution": best,
            "search_ms": round(search_ms, 4), "allgather_ms": round(gather_ms, 4),
            "search_allgather_ms": round(pair_ms, 4), "step_ms": round(step_ms, 4),
            "value": round(n_sb / (step_ms * 1e-3), 1), "value_resident_input": round(n_sb / (pair_ms * 1e-3), 1),
            "unit": "SB/s", "scaling": "strong",
            "allgather_bytes_per_rank": split.gather_bytes_in,
            "pcie_bytes_per_rank": {"pcie": Wd * Ht, "broadcast": Wd * Ht if rank == 0 else 0,
                                    "sliced": (ps.r1 - ps.r0) * Wd},
            "note": "value = SBs of the picture / the pipelined step (the current picture's 8-bit plane distributed "
                    "to every rank -- pcie: each rank's own upload; broadcast: rank 0 uploads, RCCL broadcast; "
                    "sliced: each rank uploads its H/N rows, one RCCL all-gather assembles the plane -- "
                    "its pyramid built on device, the chunk searched, the records all-gathered), max over ranks; "
                    "value_resident_input: search + all-gather with the picture already resident; the parts "
                    "timed alone"}


def cpu_leg(S, W, name, gpu_recs, gpu_sbres, cpu_seconds):
    """The reference's own ME (motion_estimation.c + its AVX2 kernels, compiled
    from source into oracle/_ref) on this host, whole-picture passes of the same
    job; the C restatement (oracle) when oracle/_ref is absent."""
    kind = "reference"
    try:
        S.load_ref().svtref_set_simd(1)
        checker = "ref"
    except Exception:
        kind, checker = "port", "oracle"
    wl = W.WORKLOADS[name]
    threads = host_cores()
    frames = W.workload_frames(name)
    pyr = {t: S.build_host_pyramid(f, "oracle") for t, f in frames.items()}
    refs = {(0, i): pyr[t] for i, t in enumerate(wl["l0"])}
    refs.update({(1, i): pyr[t] for i, t in enumerate(wl["l1"])})
    job = W.workload_job(name)
    n_sb = S.sb_total(job.width, job.height)
    t0 = time.perf_counter()
    recs, sbr = S.run_checker(job, pyr[8], refs, checker, nthreads=threads, with_sb_results=gpu_sbres is not None)
    first = time.perf_counter() - t0
    # records and (PA-ME) the per-SB results, byte for byte against the reference's
    parity = not S.compare_records(recs, gpu_recs, sbr, gpu_sbres)
    # the absolute differences the reference's searches evaluate on this job (early exits and
    # pruning included), counted by the oracle's restatement of them: the real SAD work
    absdiff = None
    try:
        ora = S.load_oracle()
        ora.svtora_absdiff.restype = C.c_uint64
        ora.svtora_absdiff.argtypes = [C.c_int]
        ora.svtora_absdiff(1)
        S.run_checker(job, pyr[8], refs, "oracle", nthreads=threads, with_sb_results=False)
        absdiff = int(ora.svtora_absdiff(1))
    except (RuntimeError, AttributeError):
        pass
    reps = max(1, int(cpu_seconds / max(first * threads, 1e-4)))
    t0 = time.perf_counter()
    for _ in range(reps):
        S.run_checker(job, pyr[8], refs, checker, nthreads=threads, with_sb_results=False)
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
             "sample": f"{reps} pass(es) over the full picture ({n_sb} SBs x {S.ref_slots(job)} refs), one SB "
                       f"per task on {threads} threads (all CPUs this process may use: affinity "
                       f"{len(os.sched_getaffinity(0))}, cgroup quota), "
                       f"{'reference AVX2 kernels' if kind == 'reference' else 'C restatement'}, "
                       f"{el:.2f} s wall, CPU: {cpu_model}"}, parity, absdiff)


if __name__ == "__main__":
    main()
