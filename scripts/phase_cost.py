"""Pass time of one k_hme build (SVTME_LIB) on a workload, HIP events on the
library stream. With the SVTME_STOP_AFTER=k builds of scripts/gpu_phase_cost.sh
the differences between consecutive builds are the phases' throughput costs.

usage: SVTME_LIB=... python3 scripts/phase_cost.py [workload] [pictures] [label]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "svt-av1-mirror_amd"))

import svtme as S  # noqa: E402
import workloads as W  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "4k_p8"
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    label = sys.argv[3] if len(sys.argv) > 3 else os.path.basename(os.environ.get("SVTME_LIB", "product"))
    wl = W.WORKLOADS[name]
    import torch

    torch.cuda.set_device(0)
    gpu = S.GpuME(0)
    syn = S.Synth(wl["w"], wl["h"])
    jobs = []
    for p in range(P):
        for t in sorted(set((8,) + tuple(wl["l0"]) + tuple(wl["l1"]))):
            gpu.upload(t + 32 * p, W.workload_frame(name, syn, t))
        jobs.append(W.workload_job(name, base=32 * p))
    n_sb = S.sb_total(wl["w"], wl["h"])
    R = S.ref_slots(jobs[0])
    bufs = [torch.zeros(n_sb * R * S.REF_RECORD_DTYPE.itemsize, dtype=torch.uint8, device="cuda") for _ in jobs]
    ptrs = [b.data_ptr() for b in bufs]
    ext = torch.cuda.ExternalStream(gpu.stream(), device=torch.device("cuda", 0))
    for _ in range(10):
        gpu.submit_batch_device(jobs, ptrs)
    gpu.sync()
    steps = 50
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(ext)
    for _ in range(steps):
        gpu.submit_batch_device(jobs, ptrs)
    ev1.record(ext)
    gpu.sync()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / steps
    print(f"{label:24s} {name} x{P}: {ms * 1e3:8.2f} us per launch, {ms * 1e3 / P:7.2f} us per picture", flush=True)
    gpu.close()


if __name__ == "__main__":
    main()
