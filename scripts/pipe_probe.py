"""Why the bench's pipelined-upload leg runs slower than upload_probe.py's
pipe_depth8 on the same box: the same 8-picture rotation after different
preludes, each in a fresh process (argv[1]): none | timing (kernel timing on
for a few launches, then off, as bench.py's kernel samples) | batch (4-picture
launches on both lanes first, as bench.py's main loop) | both. Prints ms per
picture of the pipeline and of the uploads alone."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "svt-av1-mirror_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import svtme as S  # noqa: E402
import workloads as W  # noqa: E402


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "none"
    name = "4k_p8"
    wl = W.WORKLOADS[name]
    Wd, Ht = wl["w"], wl["h"]
    gpu = S.GpuME(0)
    frames = W.workload_frames(name)
    n_sb = S.sb_total(Wd, Ht)
    dev = torch.device("cuda", 0)
    pbuf = [torch.zeros(n_sb * 4 * S.REF_RECORD_DTYPE.itemsize, dtype=torch.uint8, device=dev) for _ in range(2)]
    big = [torch.zeros(4 * n_sb * 4 * S.REF_RECORD_DTYPE.itemsize, dtype=torch.uint8, device=dev) for _ in range(2)]
    torch.cuda.synchronize()
    pinned = torch.from_numpy(np.ascontiguousarray(frames[8])).pin_memory()
    NP = 8
    bases = [930000 + 64 * k for k in range(NP)]
    jobs = []
    for b in bases:
        for t, f in frames.items():
            if t != 8:
                gpu.upload(b + t, f)
        gpu.upload_async(b + 8, pinned.data_ptr(), Wd, Ht)
        jobs.append(W.workload_job(name, base=b))
    gpu.sync()
    if mode in ("batch", "both"):
        for i in range(20):
            gpu.submit_batch_device(jobs[:4], [big[i & 1].data_ptr() + k * n_sb * 4 * S.REF_RECORD_DTYPE.itemsize
                                               for k in range(4)], lane=i & 1)
        gpu.sync()
    if mode in ("timing", "both"):
        gpu.set_timing(True)
        for i in range(10):
            gpu.submit_batch_device([jobs[0]], [pbuf[0].data_ptr()])
        gpu.sync()
        gpu.set_timing(False)
        gpu.timing_read()

    def pipe(i):
        gpu.upload_async(bases[i % NP] + 8, pinned.data_ptr(), Wd, Ht)
        gpu.submit_batch_device([jobs[i % NP]], [pbuf[i & 1].data_ptr()], lane=i & 1)
    for i in range(2 * NP):
        pipe(i)
    gpu.sync()
    reps = 80
    t0 = time.perf_counter()
    for i in range(reps):
        pipe(i)
    gpu.sync()
    pipe_ms = (time.perf_counter() - t0) / reps * 1e3
    t0 = time.perf_counter()
    for i in range(reps):
        gpu.upload_async(bases[i % NP] + 8, pinned.data_ptr(), Wd, Ht)
    gpu.sync()
    up_ms = (time.perf_counter() - t0) / reps * 1e3
    print(json.dumps({"mode": mode, "pipelined_ms": round(pipe_ms, 4), "upload_only_ms": round(up_ms, 4)}), flush=True)
    gpu.close()


if __name__ == "__main__":
    main()
