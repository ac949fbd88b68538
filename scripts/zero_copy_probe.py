"""Upload paths of one 4K picture from page-locked host memory, timed alone
(synchronous, and back to back asynchronous): (a) the default -- level 0's
interior streamed over PCIe by 128 workgroups (k_host_rows), then padded and
decimated on device; (b) the full-grid level-0 build reading the host plane
itself (svtme_picture_upload_device given the page-locked address); (c) the
DMA path (a second context with SVTME_UPLOAD_ZERO_COPY=0: one DMA into a
device staging plane, then the build). Checks the three pyramids are equal.
Prints JSON.

usage (GPU box): python3 scripts/zero_copy_probe.py
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "svt-av1-mirror_amd"))

import svtme as S  # noqa: E402
import workloads as W  # noqa: E402


def main():
    import torch

    name = "4k_p8"
    wl = W.WORKLOADS[name]
    Wd, Ht = wl["w"], wl["h"]
    gpu = S.GpuME(0)
    syn = S.Synth(Wd, Ht)
    frame = np.ascontiguousarray(W.workload_frame(name, syn, 8))
    pinned = torch.from_numpy(frame).pin_memory()
    hp = pinned.data_ptr()
    out = {"picture_bytes": int(frame.nbytes)}

    def med(fn, reps=20):
        t = []
        for k in range(reps + 3):
            t0 = time.perf_counter()
            fn(k)
            t.append(time.perf_counter() - t0)
        return round(float(np.median(t[3:])) * 1e3, 4)

    os.environ["SVTME_UPLOAD_ZERO_COPY"] = "0"
    dma = S.GpuME(0)  # (the flag is read at context creation)
    del os.environ["SVTME_UPLOAD_ZERO_COPY"]
    out["stream_sync_ms"] = med(lambda k: (gpu.upload_async(500 + (k & 7), hp, Wd, Ht), gpu.sync()))
    out["full_grid_sync_ms"] = med(lambda k: gpu.upload_device(600 + (k & 7), hp, Wd, Wd, Ht))
    out["dma_sync_ms"] = med(lambda k: (dma.upload_async(700 + (k & 7), hp, Wd, Ht), dma.sync()))
    # back-to-back asynchronous uploads of 8 rotating pictures (the copy engine's / the PCIe reads' rate)
    def burst(g, fn, n=40):
        g.sync()
        t0 = time.perf_counter()
        for k in range(n):
            fn(k)
        g.sync()
        return round((time.perf_counter() - t0) / n * 1e3, 4)
    out["stream_async_ms"] = burst(gpu, lambda k: gpu.upload_async(500 + (k & 7), hp, Wd, Ht))
    out["full_grid_async_ms"] = burst(gpu, lambda k: gpu.upload_device_async(600 + (k & 7), hp, Wd, Wd, Ht))
    out["dma_async_ms"] = burst(dma, lambda k: dma.upload_async(700 + (k & 7), hp, Wd, Ht))
    same = all(np.array_equal(gpu.download(500, lv), gpu.download(600, lv)) and
               np.array_equal(gpu.download(500, lv), dma.download(700, lv)) for lv in range(3))
    out["pyramids_equal"] = bool(same)
    print(json.dumps(out))
    dma.close()
    gpu.close()


if __name__ == "__main__":
    main()
