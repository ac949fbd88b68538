"""Experiment: the same 4K p8 work as 2 contexts (2 streams) x P/2 pictures per
launch, submitted alternately, versus 1 context x P pictures; pass time per
picture from wall-clock over many steps (device-bound)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "svt-av1-mirror_amd"))
import svtme as S  # noqa: E402
import workloads as W  # noqa: E402


def main():
    import torch

    torch.cuda.set_device(0)
    name, P, NC = "4k_p8", int(sys.argv[1]) if len(sys.argv) > 1 else 4, int(sys.argv[2]) if len(sys.argv) > 2 else 2
    wl = W.WORKLOADS[name]
    syn = S.Synth(wl["w"], wl["h"])
    n_sb = S.sb_total(wl["w"], wl["h"])
    ctxs = []
    for c in range(NC):
        g = S.GpuME(0)
        jobs = []
        for p in range(P // NC):
            for t in sorted(set((8,) + tuple(wl["l0"]) + tuple(wl["l1"]))):
                g.upload(t + 32 * p, syn.frame(t))
            jobs.append(W.workload_job(name, base=32 * p))
        R = S.ref_slots(jobs[0])
        bufs = [torch.zeros(n_sb * R * S.REF_RECORD_DTYPE.itemsize, dtype=torch.uint8, device="cuda") for _ in jobs]
        ctxs.append((g, jobs, [b.data_ptr() for b in bufs], bufs))
    for _ in range(5):
        for g, jobs, ptrs, _b in ctxs:
            g.submit_batch_device(jobs, ptrs)
    for g, *_ in ctxs:
        g.sync()
    steps = 100
    t0 = time.perf_counter()
    for _ in range(steps):
        for g, jobs, ptrs, _b in ctxs:
            g.submit_batch_device(jobs, ptrs)
    for g, *_ in ctxs:
        g.sync()
    dt = (time.perf_counter() - t0) / steps
    print(f"{NC} context(s) x {P // NC} pictures: {dt * 1e6 / P:.2f} us per picture", flush=True)
    for g, *_ in ctxs:
        g.close()


if __name__ == "__main__":
    main()
