"""Upload-pipeline probe (4K p8): where does the asynchronous upload leg lose time?

Each variant runs `reps` steps after a warm-up and prints ms per picture:
  upload_only     svtme_picture_upload_async of a pinned 4K plane, 4 rotating pictures
  me_only         one 4K p8 job per launch on lane 0, pictures resident
  pipe_lane0      upload_async(picture i) + its job on lane 0 (bench.py's `pipelined`)
  pipe_lanes      the same, jobs alternating lanes 0 / 1
  pipe_depth8     8 rotating pictures instead of 4
  torch_h2d       a plain pinned -> device copy of the same bytes on a side stream (PCIe rate)
  torch_h2d_me    the same copies on a side stream while lane 0 runs the ME steps
Run it under `rocprofv3 --kernel-trace --memory-copy-trace` to see the timeline.
"""
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
    name = "4k_p8"
    wl = W.WORKLOADS[name]
    Wd, Ht = wl["w"], wl["h"]
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    gpu = S.GpuME(0)
    frames = W.workload_frames(name)
    for t, f in frames.items():
        gpu.upload(t, f)
    frame = frames[8]
    pinned = torch.from_numpy(np.ascontiguousarray(frame)).pin_memory()
    n_sb = S.sb_total(Wd, Ht)
    R = 4
    out = {}
    dev = torch.device("cuda", 0)
    pbuf = [torch.zeros(n_sb * R * S.REF_RECORD_DTYPE.itemsize, dtype=torch.uint8, device=dev) for _ in range(2)]

    def jobs_for(base, n):  # picture set k at base + 64 k, its references resident (realistic distances)
        js = []
        for k in range(n):
            b = base + 64 * k
            for t, f in frames.items():
                if t != 8:
                    gpu.upload(b + t, f)
            js.append(W.workload_job(name, base=b))
        return js

    def timed(fn, n=reps, warm=8):
        for i in range(warm):
            fn(i)
        gpu.sync()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            fn(warm + i)
        gpu.sync()
        torch.cuda.synchronize()
        return round((time.perf_counter() - t0) / n * 1e3, 4)

    pj4 = jobs_for(910000, 4)
    pj8 = jobs_for(920000, 8)
    for k in range(8):  # make the rotating pictures resident once
        gpu.upload_async(920000 + 64 * k + 8, pinned.data_ptr(), Wd, Ht)
    for k in range(4):
        gpu.upload_async(910000 + 64 * k + 8, pinned.data_ptr(), Wd, Ht)
    gpu.sync()
    jme = W.workload_job(name)

    out["upload_only"] = timed(lambda i: gpu.upload_async(910000 + 64 * (i & 3) + 8, pinned.data_ptr(), Wd, Ht))
    out["me_only"] = timed(lambda i: gpu.submit_batch_device([jme], [pbuf[0].data_ptr()]))
    out["me_only_lanes"] = timed(lambda i: gpu.submit_batch_device([jme], [pbuf[i & 1].data_ptr()], lane=i & 1))

    def pipe0(i):
        gpu.upload_async(910000 + 64 * (i & 3) + 8, pinned.data_ptr(), Wd, Ht)
        gpu.submit_batch_device([pj4[i & 3]], [pbuf[0].data_ptr()])
    out["pipe_lane0"] = timed(pipe0)

    def pipel(i):
        gpu.upload_async(910000 + 64 * (i & 3) + 8, pinned.data_ptr(), Wd, Ht)
        gpu.submit_batch_device([pj4[i & 3]], [pbuf[i & 1].data_ptr()], lane=i & 1)
    out["pipe_lanes"] = timed(pipel)

    def pipe8(i):
        gpu.upload_async(920000 + 64 * (i & 7) + 8, pinned.data_ptr(), Wd, Ht)
        gpu.submit_batch_device([pj8[i & 7]], [pbuf[i & 1].data_ptr()], lane=i & 1)
    out["pipe_depth8"] = timed(pipe8)

    side = torch.cuda.Stream(device=dev)
    dst = torch.empty(frame.size, dtype=torch.uint8, device=dev)
    src = pinned.view(-1)

    def h2d(i):
        with torch.cuda.stream(side):
            dst.copy_(src, non_blocking=True)
    out["torch_h2d"] = timed(h2d)

    def h2d_me(i):
        with torch.cuda.stream(side):
            dst.copy_(src, non_blocking=True)
        gpu.submit_batch_device([jme], [pbuf[0].data_ptr()])
    out["torch_h2d_me"] = timed(h2d_me)
    out["picture_bytes"] = int(frame.nbytes)
    out["reps"] = reps
    print(json.dumps(out), flush=True)
    gpu.close()


if __name__ == "__main__":
    main()
