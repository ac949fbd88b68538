"""Packed host output (svtme_submit_picture_packed_async, include/svtme.h
svtme_pack_layout): the bytes the encoder glue scatters (integration/
svtme_svt_glue.c) equal the numpy restatement of the documented layout
(svtme.pack_outputs) over the job's full outputs.

CPU: the oracle job API (oracle/liboraclejob.so, the encoder tests' backend).
GPU: k_pack behind the ticket API of libsvtme.so, several jobs in flight on
both submission lanes, the ticket limit, and jobs after svtme_reserve.
"""
import pytest

import svtme as S

W, H = 640, 360
# (n_pus, max_cand, max_refs, full_records, sb_results): PA-ME allocations of
# pcs.c:91-117 (85 / 21 / 5 PUs; 2+1 refs: 3 MVs, 3 + 2 + 1 = 6 candidates) and TF-ME's
LAYOUTS = [(85, 6, 3, 0, 1), (21, 6, 3, 0, 1), (5, 23, 7, 0, 1), (85, 6, 3, 1, 1), (0, 0, 0, 1, 0)]


def _layout(t):
    L = S.PackLayout()
    L.n_pus, L.max_cand, L.max_refs, L.full_records, L.sb_results = t
    return L


def _setup(api, base):
    frames = S.test_frames("pan", W, H, [6, 7, 8, 9])
    for t, f in frames.items():
        api.upload(base + t, f)
    ctrl = S.derive_controls(8, 35, S.input_resolution_of(W, H), 1)
    return S.make_job(W, H, ctrl, base + 8, (base + 7, base + 6), (base + 9,), temporal_layer_index=1,
                      ref_count_used=(2, 1))


def test_reserve_arguments_oracle_backend():
    api = S.GpuME(0, lib=S.load_oracle_job())
    api.reserve(W, H, 8, 4)
    for bad in ((0, H, 8, 4), (W, H, 0, 4), (W, H, 9, 4), (W, H, 8, S.MAX_TICKETS + 1)):
        with pytest.raises(RuntimeError):
            api.reserve(*bad)
    api.close()


def test_packed_layout_oracle_backend():
    api = S.GpuME(0, lib=S.load_oracle_job())
    job = _setup(api, 0)
    recs, sbr = api.submit(job)
    for t in LAYOUTS:
        L = _layout(t)
        got = api.submit_packed(job, L)
        assert got == S.pack_outputs(recs, sbr if L.sb_results else None, L), t
    api.close()


@pytest.mark.gpu
def test_packed_output_gpu(gpu):
    job = _setup(gpu, 7000)
    recs, sbr = gpu.submit(job)
    for t in LAYOUTS:
        L = _layout(t)
        assert gpu.submit_packed(job, L, lane=t[0] & 1) == S.pack_outputs(recs, sbr if L.sb_results else None, L), t
    # several jobs in flight on both lanes, retired out of order
    L = _layout(LAYOUTS[0])
    exp = S.pack_outputs(recs, sbr, L)
    pend = [gpu.submit_packed(job, L, lane=k & 1, wait=False) for k in range(6)]
    for p in reversed(pend):
        assert gpu.wait_packed(*p) == exp
    # at most SVTME_MAX_TICKETS outstanding: one thread holding them all is refused the
    # next one (nobody retires a ticket within the grace period), the context keeps serving
    pend = [gpu.submit_packed(job, L, lane=k & 1, wait=False) for k in range(S.MAX_TICKETS)]
    with pytest.raises(RuntimeError, match="outstanding"):
        gpu.submit_packed(job, L, wait=False)
    for p in pend:
        assert gpu.wait_packed(*p) == exp
    assert gpu.submit_packed(job, L) == exp
    # more submitting threads than ticket slots (the reference's up to 25 ME threads plus
    # TF threads, each with a job in flight): a submission finding every slot taken waits
    # for another thread's svtme_ticket_wait instead of failing
    import threading

    errs, done = [], []

    def worker(k):
        try:
            for _ in range(3):
                if gpu.submit_packed(job, L, lane=k & 1) != exp:
                    errs.append(f"thread {k}: packed bytes differ")
            done.append(k)
        except Exception as e:  # noqa: BLE001
            errs.append(f"thread {k}: {e}")
    th = [threading.Thread(target=worker, args=(k,)) for k in range(S.MAX_TICKETS + 16)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=60)
    assert not errs and len(done) == S.MAX_TICKETS + 16, errs[:3]
    # reserved for a larger picture (every lane's scratch, the first tickets' buffers):
    # the same bytes, and a picture beyond the reservation still grows what it needs
    gpu.reserve(W, H // 2, 3, 2)
    gpu.reserve(2 * W, 2 * H, 8, 6)
    for t in LAYOUTS:
        L = _layout(t)
        assert gpu.submit_packed(job, L, lane=1 - (t[0] & 1)) == S.pack_outputs(recs, sbr if L.sb_results else None, L), t
    for bad in ((0, H, 8, 4), (W, H, 9, 4), (W, H, 8, S.MAX_TICKETS + 1)):
        with pytest.raises(RuntimeError):
            gpu.reserve(*bad)
    for t in (6, 7, 8, 9):
        gpu.release(7000 + t)
