"""Where a served picture job's latency goes: the glue's call pattern
(svtme_submit_picture_packed_async of one 4K p8 PA job into a page-locked
buffer, then svtme_ticket_wait_timed), timed host-side per call, with a gap
between jobs like the encoder's (~2 ms of CPU work between pictures) and
back to back.

usage (GPU box): python3 scripts/submit_probe.py [jobs] [gap_ms ...]
Prints JSON: per gap, p50 / p90 of the submit call, the wait, the whole job,
and the library's GPU / copy times.
"""
import ctypes as C
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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    gaps = [float(x) for x in sys.argv[2:]] or [2.0, 0.0]
    name = "4k_p8"
    wl = W.WORKLOADS[name]
    gpu = S.GpuME(0)
    syn = S.Synth(wl["w"], wl["h"])
    for t in sorted(set((8,) + tuple(wl["l0"]) + tuple(wl["l1"]))):
        gpu.upload(t, W.workload_frame(name, syn, t))
    job = W.workload_job(name)
    L = S.PackLayout()
    L.n_pus, L.max_cand, L.max_refs, L.full_records, L.sb_results = S.PU_COUNT, 23, 7, 0, 1
    nbytes = S.sb_total(wl["w"], wl["h"]) * S.packed_sb_bytes(L, S.ref_slots(job))
    gpu.reserve(wl["w"], wl["h"], 4, 8)
    bufs = [gpu.lib.svtme_host_alloc(nbytes) for _ in range(2)]
    lib = gpu.lib
    lib.svtme_submit_picture_packed_async.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(S.Job),
                                                      C.POINTER(S.PackLayout), C.c_void_p, C.POINTER(C.c_uint64)]
    lib.svtme_submit_picture_packed_async.restype = C.c_int32
    lib.svtme_ticket_wait_timed.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(C.c_float), C.POINTER(C.c_float)]
    lib.svtme_ticket_wait_timed.restype = C.c_int32
    out = {"workload": name, "packed_bytes": nbytes, "jobs": n, "runs": []}
    for gap in gaps:
        rec = []
        for i in range(n + 5):
            if gap:
                t_end = time.perf_counter() + gap * 1e-3
                while time.perf_counter() < t_end:
                    pass
            tk = C.c_uint64()
            g, cp = C.c_float(), C.c_float()
            t0 = time.perf_counter()
            gpu._check(lib.svtme_submit_picture_packed_async(gpu.ctx, i & 1, C.byref(job), C.byref(L), bufs[i & 1],
                                                             C.byref(tk)), "submit")
            t1 = time.perf_counter()
            gpu._check(lib.svtme_ticket_wait_timed(gpu.ctx, tk.value, C.byref(g), C.byref(cp)), "wait")
            t2 = time.perf_counter()
            rec.append(((t1 - t0) * 1e3, (t2 - t1) * 1e3, (t2 - t0) * 1e3, g.value, cp.value))
        a = np.array(rec[5:])
        q = lambda col, p: round(float(np.percentile(a[:, col], p)), 4)  # noqa: E731
        out["runs"].append({"gap_ms": gap, **{f"{k}_p50": q(c, 50) for c, k in enumerate(("submit", "wait", "job", "gpu", "copy"))},
                            **{f"{k}_p90": q(c, 90) for c, k in enumerate(("submit", "wait", "job", "gpu", "copy"))},
                            "served_sb_per_s": round(S.sb_total(wl["w"], wl["h"]) / (float(np.mean(a[:, 2])) * 1e-3), 1)})
    # TF windows: n (central, reference) pairs in one svtme_submit_pictures_packed_async, as the glue's
    # tf_window submits them (whole records, no SB results)
    for t in (4, 5, 6, 9, 10, 11, 12):
        if t not in (7, 8):
            gpu.upload(t, W.workload_frame(name, syn, t))
    Lt = S.PackLayout()
    Lt.n_pus, Lt.max_cand, Lt.max_refs, Lt.full_records, Lt.sb_results = 0, 0, 0, 1, 0
    lib.svtme_submit_pictures_packed_async.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(S.Job),
                                                       C.POINTER(S.PackLayout), C.POINTER(C.c_void_p),
                                                       C.POINTER(C.c_uint64)]
    lib.svtme_submit_pictures_packed_async.restype = C.c_int32
    tfbytes = S.sb_total(wl["w"], wl["h"]) * S.packed_sb_bytes(Lt, 1)
    tbufs = [lib.svtme_host_alloc(tfbytes) for _ in range(8)]
    out["tf_windows"] = []
    for npairs in (1, 2, 4, 8):
        base = W.workload_job("4k_tf_p8")
        refs = [4, 5, 6, 7, 9, 10, 11, 12][:npairs]
        jobs = []
        for r in refs:
            j = W.workload_job("4k_tf_p8")
            j.ref_picture_number[0][0] = r
            jobs.append(j)
        arr_j = (S.Job * npairs)(*jobs)
        arr_l = (S.PackLayout * npairs)(*([Lt] * npairs))
        arr_p = (C.c_void_p * npairs)(*tbufs[:npairs])
        rec = []
        for i in range(25):
            tks = (C.c_uint64 * npairs)()
            t0 = time.perf_counter()
            gpu._check(lib.svtme_submit_pictures_packed_async(gpu.ctx, i & 1, npairs, arr_j, arr_l, arr_p, tks), "tf submit")
            t1 = time.perf_counter()
            for k in range(npairs):
                gpu._check(lib.svtme_ticket_wait(gpu.ctx, tks[k]), "tf wait")
            t2 = time.perf_counter()
            rec.append(((t1 - t0) * 1e3, (t2 - t0) * 1e3))
        a = np.array(rec[5:])
        out["tf_windows"].append({"pairs": npairs, "submit_p50": round(float(np.median(a[:, 0])), 4),
                                  "job_p50": round(float(np.median(a[:, 1])), 4)})
        del base
    for b in tbufs:
        lib.svtme_host_free(b)
    print(json.dumps(out))
    for b in bufs:
        lib.svtme_host_free(b)
    gpu.close()


if __name__ == "__main__":
    main()
