"""Upload cost from encoder-like host memory (4K 8-bit plane with the encoder's
72-sample padding, stride 3984): pageable buffers never uploaded before, the
same pageable buffer again, hipHostRegister of a fresh buffer and the upload
from it, a host memcpy into page-locked staging. Prints ms per picture."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "svt-av1-mirror_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import svtme as S  # noqa: E402


def main():
    W, H, PAD = 3840, 2160, 72
    stride = W + 2 * PAD
    rows = H + 2 * PAD
    gpu = S.GpuME(0)
    rt = torch.cuda.cudart()
    n = 12
    bufs = [np.random.default_rng(k).integers(0, 256, (rows, stride), dtype=np.uint8) for k in range(n)]
    out = {}

    def up(buf, pn):
        y = buf[PAD:, PAD:]
        gpu.upload_async(pn, y.ctypes.data, W, H, stride)
        gpu.sync()

    up(bufs[0], 1)  # warm-up
    t = []
    for k in range(1, n // 2):
        t0 = time.perf_counter()
        up(bufs[k], 1)
        t.append(time.perf_counter() - t0)
    out["pageable_fresh_ms"] = round(1e3 * float(np.median(t)), 4)
    t = []
    for k in range(6):
        t0 = time.perf_counter()
        up(bufs[1], 1)
        t.append(time.perf_counter() - t0)
    out["pageable_reused_ms"] = round(1e3 * float(np.median(t)), 4)
    reg, upr = [], []
    for k in range(n // 2, n):
        b = bufs[k]
        t0 = time.perf_counter()
        err = rt.cudaHostRegister(b.ctypes.data, b.nbytes, 0)
        reg.append(time.perf_counter() - t0)
        assert int(err) == 0, err
        t0 = time.perf_counter()
        up(b, 1)
        upr.append(time.perf_counter() - t0)
    out["register_ms"] = round(1e3 * float(np.median(reg)), 4)
    out["registered_upload_ms"] = round(1e3 * float(np.median(upr)), 4)
    t = []
    for k in range(n // 2, n):
        t0 = time.perf_counter()
        up(bufs[k], 1)
        t.append(time.perf_counter() - t0)
    out["registered_upload_again_ms"] = round(1e3 * float(np.median(t)), 4)
    for k in range(n // 2, n):
        rt.cudaHostUnregister(bufs[k].ctypes.data)
    pinned = torch.empty(rows * stride, dtype=torch.uint8).pin_memory().numpy().reshape(rows, stride)
    t = []
    for k in range(1, n // 2):
        t0 = time.perf_counter()
        np.copyto(pinned, bufs[k])
        up(pinned, 1)
        t.append(time.perf_counter() - t0)
    out["memcpy_to_pinned_then_upload_ms"] = round(1e3 * float(np.median(t)), 4)
    print(json.dumps(out), flush=True)
    gpu.close()


if __name__ == "__main__":
    main()
