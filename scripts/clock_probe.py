"""Why the first launches of a fresh process run slower: the in-kernel clock of
k_hme over time, from a diagnostic build (-DSVTME_CLOCKBINS).

Build (container):  bash scripts/build_diag_lib.sh clk -DSVTME_CLOCKBINS
Run (GPU box):      python3 scripts/clock_probe.py [steps] [idle_ms]

Replays bench.py's timed loop in a fresh process (the workload's pictures
uploaded, then steps of 4 pictures per launch on the two submission lanes, no
warm-up), optionally pausing idle_ms first. Thread 0 of every k_hme workgroup
adds its shader cycles (s_memtime) and its 100 MHz real-time ticks
(s_memrealtime) into the ~82 us bin of its start time, so per bin:
clock = cycles / ticks x 100 MHz (the MI355X_MICROARCH.md item-6 method, the
median over workgroups replaced by the cycle-weighted mean of the bin) and the
mean workgroup duration in ns. Host-side: the wall time of every block of 20
steps (a fence after each block; the bench's own timed region is 20 steps).
Prints JSON to stdout.
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("SVTME_LIB", os.path.join(ROOT, "svt-av1-mirror_amd", "libsvtme_clk.so"))
sys.path.insert(0, os.path.join(ROOT, "svt-av1-mirror_amd"))

import svtme as S  # noqa: E402
import workloads as W  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    idle_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
    name, P, block = "4k_p8", 4, 20
    wl = W.WORKLOADS[name]
    import torch

    torch.cuda.set_device(0)
    gpu = S.GpuME(0)
    syn = S.Synth(wl["w"], wl["h"])
    offs = sorted(set((0,) + tuple(t - 8 for t in wl["l0"]) + tuple(t - 8 for t in wl["l1"])))
    jobs = []
    for p in range(P):
        t0 = 8 + 32 * p
        for o in offs:
            gpu.upload(t0 + o, W.workload_frame(name, syn, t0 + o))
        jobs.append(W.workload_job(name, base=32 * p))
    n_sb = S.sb_total(wl["w"], wl["h"])
    R = S.ref_slots(jobs[0])
    rec = S.REF_RECORD_DTYPE.itemsize
    bufs = [torch.zeros(P * n_sb * R * rec, dtype=torch.uint8, device="cuda") for _ in range(2)]
    gpu.sync()
    torch.cuda.synchronize()
    if idle_ms:
        time.sleep(idle_ms * 1e-3)
    blocks = []
    t_start = time.perf_counter()
    for b0 in range(0, steps, block):
        t0 = time.perf_counter()
        for i in range(b0, min(steps, b0 + block)):
            gpu.submit_batch_device(jobs, [bufs[i & 1].data_ptr() + p * n_sb * R * rec for p in range(P)], lane=i & 1)
        gpu.sync()
        blocks.append(round((time.perf_counter() - t0) * 1e3 / block, 4))
    total = time.perf_counter() - t_start
    lib = S.load_product()
    fn = lib.svtme_debug_clock_bins
    fn.argtypes = [C.c_void_p]
    fn.restype = C.c_int
    bins = np.zeros((4096, 3), np.uint64)
    assert fn(bins.ctypes.data) == 0
    bins = bins.astype(np.float64)
    used = np.nonzero(bins[:, 2])[0]
    # unwrap: the run starts after the longest run of empty bins
    occ = bins[:, 2] > 0
    gaps = (np.roll(used, -1) - used) % 4096
    start = int(used[(int(np.argmax(gaps)) + 1) % len(used)]) if len(used) > 1 else int(used[0])
    order = np.roll(np.arange(4096), -start)
    series = []
    for k in order:
        if not occ[k]:
            continue
        cyc, tick, n = bins[k]
        series.append({"bin": int((k - start) % 4096), "t_us": round(((k - start) % 4096) * 81.92, 1),
                       "ghz": round(cyc / tick * 0.1, 4), "wg_ns": round(tick * 10.0 / n, 1), "wgs": int(n)})
    ghz = [s["ghz"] for s in series]
    out = {"workload": name, "pictures_per_launch": P, "steps": steps, "idle_ms_before": idle_ms,
           "ms_per_step_blocks_of_20": blocks, "total_s": round(total, 4),
           "clock_ghz_first5_bins": ghz[:5], "clock_ghz_last5_bins": ghz[-5:],
           "clock_ghz_median_first_10pct": float(np.median(ghz[: max(1, len(ghz) // 10)])),
           "clock_ghz_median_last_50pct": float(np.median(ghz[len(ghz) // 2:])),
           "bins": series}
    print(json.dumps(out))
    gpu.close()


if __name__ == "__main__":
    main()
