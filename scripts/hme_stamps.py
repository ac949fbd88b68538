"""Per-phase timing of k_hme from a diagnostic build (-DSVTME_STAMPS).

Build (container):  bash scripts/build_diag_lib.sh stamp -DSVTME_STAMPS
Run (GPU box):      python3 scripts/hme_stamps.py [workload] [pictures] [records]
                    (records: the records alone; default the whole output, as bench.py times it)

Thread 0 of every k_hme workgroup stamps the shader clock at 7 points: start,
after A0 (zz), after the A1 table, after A1 tiles, after D + L1 table, after
the L1 tiles, end. Prints per-phase cycle statistics and the launch span.
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("SVTME_LIB", os.path.join(ROOT, "svt-av1-mirror_amd", "libsvtme_stamp.so"))
sys.path.insert(0, os.path.join(ROOT, "svt-av1-mirror_amd"))

import svtme as S  # noqa: E402
import workloads as W  # noqa: E402

PHASES = ["A0 (job, zz, A1 table)", "zz decisions", "A1 tiles", "D + L1 table", "L1 (+L2) tiles", "final centre",
          "full-pel", "E (prune, records, SB results)"]


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "4k_p8"
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    wl = W.WORKLOADS[name]
    import torch

    torch.cuda.set_device(0)  # torch first (as bench.py), then the library's context
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
    sbb = None if (len(sys.argv) > 3 and sys.argv[3] == "records") else \
        [torch.zeros(n_sb * S.SB_RESULT_DTYPE.itemsize, dtype=torch.uint8, device="cuda") for _ in jobs]
    for _ in range(5):
        gpu.submit_batch_device(jobs, [b.data_ptr() for b in bufs], None if sbb is None else [b.data_ptr() for b in sbb])
    gpu.sync()
    lib = S.load_product()
    nb = n_sb * P
    st = np.zeros((nb, 32), np.uint64)
    fn = lib.svtme_debug_hme_stamps
    fn.argtypes = [C.c_void_p, C.c_uint32]
    fn.restype = C.c_int
    assert fn(st.ctypes.data, nb) == 0
    st = st.astype(np.int64)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.save(os.path.join(ROOT, "gpurun_out", f"stamps_{name}_x{P}.npy"), st)
    rt, ids, st_w = st[:, 8:10], st[:, 10:12], st[:, 12:16]
    wv = st[:, 24:32]  # per wavefront: phase-0 work done, full-pel records done
    if wv.any():
        for w in range(4):
            print(f"  wave {w}: phase-0 work done at mean {np.mean(wv[:, w] - st[:, 0]):7.0f} cycles after start; "
                  f"full-pel records done {np.mean(wv[:, 4 + w] - st[:, 16]):7.0f} after the final centre")
    fp = st[:, 22:24]  # wave 0's record: search area (check_00_center, probe) done, search done
    if fp.all():
        print(f"  wave 0 full-pel: area + probe {np.mean(fp[:, 0] - st[:, 16]):7.0f} cycles after the final centre, "
              f"search {np.mean(fp[:, 1] - fp[:, 0]):7.0f}, keys {np.mean(wv[:, 4] - fp[:, 1]):7.0f}")
    esub = st[:, [6, 17, 18, 19, 20, 21, 7]]  # stage E: decode + prune, records, image zero, SB results
    st = np.concatenate([st[:, :6], st[:, 16:17], st[:, 6:8]], axis=1)  # ... L1, centre, full-pel, E
    if not st[:, 8].any():  # HME-only build: the last stamp is 6
        st = st[:, :6]
    d = np.diff(st, axis=1)
    print(f"{name} x{P}: {nb} workgroups, per-WG total mean {np.mean(st[:, -1] - st[:, 0]):.0f} cycles "
          f"(stamps are per-XCD clocks: no launch span)")
    for k, ph in enumerate(PHASES[: d.shape[1]]):
        v = d[:, k]
        print(f"  {ph:14s} mean {v.mean():8.0f}  p50 {np.median(v):8.0f}  p90 {np.percentile(v, 90):8.0f}  max {v.max():8.0f}")
    if esub[:, 1:].all():
        de = np.diff(esub, axis=1)
        for k, ph in enumerate(["E: decode + me_prune_ref", "E: records", "E: zero SB image", "E: candidate arrays",
                                "E: SB results out", "E: end"]):
            v = de[:, k]
            print(f"    {ph:24s} mean {v.mean():8.0f}  p50 {np.median(v):8.0f}  p90 {np.percentile(v, 90):8.0f}")
    # the 100 MHz real-time clock is chip-wide: launch span, start / end spread
    t0 = rt[:, 0].min()
    s0, s1 = (rt[:, 0] - t0) * 10.0, (rt[:, 1] - t0) * 10.0  # ns
    print(f"  real time: span {s1.max():.0f} ns; WG start p50 {np.median(s0):.0f} p90 {np.percentile(s0, 90):.0f} "
          f"max {s0.max():.0f}; WG end p10 {np.percentile(s1, 10):.0f} p50 {np.median(s1):.0f} max {s1.max():.0f}; "
          f"WG duration p50 {np.median(s1 - s0):.0f} max {(s1 - s0).max():.0f}")
    xcc = ids[:, 0] & 0xF
    for x in range(8):
        m = xcc == x
        if m.any():
            print(f"  XCC {x}: {m.sum():4d} WGs (blockIdx%8 = {sorted(set((np.nonzero(m)[0] % 8).tolist()))[:4]}) "
                  f"start max {s0[m].max():.0f} end max {s1[m].max():.0f} ns")
    cu = (ids[:, 1] >> 8) & 0xF
    se = (ids[:, 1] >> 13) & 0x7
    key = xcc * 1000 + se * 100 + cu
    _, cnt = np.unique(key, return_counts=True)
    simd = (st_w >> 4) & 3
    print("  SIMD of waves 0-3, share of WGs with wave w on SIMD (w + r) & 3, r = 0..3:",
          [[round(float(np.mean(simd[:, w] == ((w + r) & 3))), 2) for r in range(4)] for w in range(4)])
    print(f"  distinct CUs {len(cnt)}; WGs per CU min {cnt.min()} p50 {np.median(cnt):.0f} max {cnt.max()}")
    gpu.close()


if __name__ == "__main__":
    main()
