"""GPU parity: the HIP picture job (libsvtme.so) vs the CPU oracle, bit-exact.

The oracle is itself pinned to the reference (tests/test_oracle_vs_ref.py and
tests/golden/). Cases mirror the reference's orchestration shapes: base and
non-base layers, 1..4 refs per list, P and B pictures, partial SBs at the
right/bottom edges, presets 4/6/8/12 (check_00_center, HME-L2, pre-HME with
line skipping, 8x8-variance resize), flat/saturated/noise content for ties.
"""
import ctypes as C
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def run_case(S, gpu, kind, w, h, mode, tl, l0, l1, cur=8, gm=False, is_ref=True, e8=None, sb_begin=0, sb_count=0,
             only_l_bwd=True, ctrl_set=None):
    frames = S.test_frames(kind, w, h, sorted(set([cur] + list(l0) + list(l1))))
    res = S.input_resolution_of(w, h)
    ctrl = S.derive_controls(mode, 35, res, tl)
    for k, v in (ctrl_set or {}).items():
        setattr(ctrl, k, v)
    job = S.make_job(w, h, ctrl, cur, l0, l1, temporal_layer_index=tl, is_ref=is_ref,
                     enable_me_8x8=(res <= S.RES_720P) if e8 is None else e8,
                     ref_count_used=(max(len(l0), 1), len(l1)), gm_enabled=gm, sb_begin=sb_begin, sb_count=sb_count,
                     only_l_bwd=only_l_bwd)
    for t, f in frames.items():
        gpu.upload(1000 + t, f)
    job.picture_number = 1000 + cur
    for i, t in enumerate(l0):
        job.ref_picture_number[0][i] = 1000 + t
    for i, t in enumerate(l1):
        job.ref_picture_number[1][i] = 1000 + t
    recs, sbr = gpu.submit(job)
    pyr = {t: S.build_host_pyramid(f, "oracle") for t, f in frames.items()}
    refs = {}
    for i, t in enumerate(l0):
        refs[(0, i)] = pyr[t]
    for i, t in enumerate(l1):
        refs[(1, i)] = pyr[t]
    ojob = S.make_job(w, h, ctrl, cur, l0, l1, temporal_layer_index=tl, is_ref=is_ref,
                      enable_me_8x8=(res <= S.RES_720P) if e8 is None else e8,
                      ref_count_used=(max(len(l0), 1), len(l1)), gm_enabled=gm, sb_begin=sb_begin,
                      sb_count=sb_count, only_l_bwd=only_l_bwd)
    orecs, osbr = S.run_checker(ojob, pyr[cur], refs, "oracle", nthreads=8)
    for t in frames:
        gpu.release(1000 + t)
    return S.compare_records(orecs, recs, osbr, sbr)


CASES = [
    ("pan", 640, 360, 8, 1, (7, 6), (9, 10)),
    ("pan", 640, 360, 8, 0, (7, 6, 5), (9, 10)),
    ("pan", 640, 360, 12, 0, (7,), ()),
    ("pan", 640, 360, 6, 1, (7,), (9,)),
    ("pan", 640, 360, 4, 2, (7, 6), (9,)),
    ("pan", 426, 240, 8, 2, (7, 6), (9,)),
    ("pan", 1000, 562, 8, 1, (7, 6), (9, 10)),
    ("pan", 72, 40, 8, 1, (7, 6), (9, 10)),
    ("pan", 136, 8, 6, 1, (7,), (9,)),
    ("pan", 640, 360, 8, 3, (7, 6, 4, 3), (9, 10, 12)),
    ("noise", 320, 192, 8, 1, (7, 6), (9, 10)),
    ("flat", 320, 192, 8, 1, (7, 6), (9, 10)),
    ("flat", 320, 192, 4, 1, (7,), (9,)),
    ("sat", 320, 192, 6, 1, (7, 6), (9,)),
    ("stripes", 320, 192, 8, 1, (7, 6), (9, 10)),
    ("stripes", 320, 192, 6, 0, (7, 6, 5), (9, 10)),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0]}-{c[1]}x{c[2]}-p{c[3]}-tl{c[4]}-{len(c[5])}+{len(c[6])}")
def test_picture_parity(svtme, gpu, case):
    errs = run_case(svtme, gpu, *case)
    assert not errs, errs[:5]


# The per-SB candidate arrays (finish_sb: construct_me_candidate_array*, motion_estimation.c:
# 2532-2835) off the default path: every bipred pair, L0-L0 and L1-L1 candidates (only_l_bwd 0,
# 4 + 3 references), the unipred pruning threshold on and off, the best-unipred-only rule of the
# one-reference-per-list case, and the single-reference case
SB_CASES = [
    ("pan", 640, 360, 8, 3, (7, 6, 4, 3), (9, 10, 12), False, None),
    ("noise", 320, 192, 8, 1, (7, 6), (9, 10), False, None),
    ("stripes", 320, 192, 8, 1, (7, 6, 5), (9,), False, {"prune_me_candidates_th": 0}),
    ("pan", 320, 192, 8, 1, (7, 6), (9, 10, 11), False, {"prune_me_candidates_th": 5}),
    ("noise", 320, 192, 8, 1, (7,), (9,), False, {"use_best_unipred_cand_only": 1}),
    ("pan", 320, 192, 8, 1, (7,), (9,), True, {"use_best_unipred_cand_only": 0}),
    ("flat", 320, 192, 8, 1, (7,), (), False, None),
]


@pytest.mark.parametrize("case", SB_CASES, ids=lambda c: f"{c[0]}-{len(c[5])}+{len(c[6])}-lbwd{int(c[7])}-{c[8]}")
def test_candidate_arrays_parity(svtme, gpu, case):
    kind, w, h, mode, tl, l0, l1, lbwd, cs = case
    errs = run_case(svtme, gpu, kind, w, h, mode, tl, l0, l1, gm=True, only_l_bwd=lbwd, ctrl_set=cs)
    assert not errs, errs[:5]


def test_gm_parity(svtme, gpu):
    assert not run_case(svtme, gpu, "pan", 640, 360, 4, 1, (7, 6), (9,), gm=True)
    assert not run_case(svtme, gpu, "pan", 1280, 720, 8, 1, (7,), (9,), gm=True)


def test_sb_range_parity(svtme, gpu):
    # a shard of the picture (the multi-GPU band) must equal the same SBs of the full job
    assert not run_case(svtme, gpu, "pan", 640, 360, 8, 1, (7, 6), (9, 10), sb_begin=17, sb_count=23)


def test_pyramid_parity(svtme, gpu):
    S = svtme
    for (w, h) in ((640, 360), (1000, 562), (72, 40)):
        f = S.Synth(w, h).frame(3)
        gpu.upload(77, f)
        p = S.build_host_pyramid(f, "oracle")
        for lv, name in enumerate(("full", "quarter", "sixteenth")):
            assert np.array_equal(gpu.download(77, lv), getattr(p, name)), (w, h, name)
        gpu.release(77)


def test_zero_copy_upload_parity(svtme, gpu):
    """Uploads from page-locked memory (the GPU streams the host plane itself,
    k_host_rows) equal the reference's pyramid like the DMA path's, at widths
    that leave a partial 16-byte chunk per row, with the plane at an offset
    inside a larger pinned buffer and a padded stride, synchronous and
    asynchronous; an unaligned pinned source (odd byte offset) falls back to
    the DMA and still matches; so does a context with SVTME_UPLOAD_ZERO_COPY=0."""
    import os

    import torch

    S = svtme
    dma_ctx = None
    try:
        os.environ["SVTME_UPLOAD_ZERO_COPY"] = "0"
        dma_ctx = S.GpuME(0)
    finally:
        del os.environ["SVTME_UPLOAD_ZERO_COPY"]
    try:
        for (w, h, pad, off) in ((426, 240, 2, 0), (1000, 562, 72, 4 * 1000 + 8), (72, 40, 12, 0),
                                 (328, 200, 5, 1)):
            f = S.Synth(w, h).frame(5)
            stride = w + pad
            buf = torch.zeros(off + stride * h + 64, dtype=torch.uint8).pin_memory()
            view = buf[off:off + stride * h].view(h, stride)
            view[:, :w] = torch.from_numpy(np.ascontiguousarray(f))
            ptr = buf.data_ptr() + off
            ref = S.build_host_pyramid(f, "oracle")
            gpu.upload_async(78, ptr, w, h, stride)
            gpu._check(gpu.lib.svtme_picture_upload(gpu.ctx, 79, ptr, stride, w, h), "svtme_picture_upload")
            dma_ctx.upload_async(80, ptr, w, h, stride)
            gpu.sync()
            dma_ctx.sync()
            for lv, name in enumerate(("full", "quarter", "sixteenth")):
                exp = getattr(ref, name)
                assert np.array_equal(gpu.download(78, lv), exp), (w, h, pad, off, name, "async")
                assert np.array_equal(gpu.download(79, lv), exp), (w, h, pad, off, name, "sync")
                assert np.array_equal(dma_ctx.download(80, lv), exp), (w, h, pad, off, name, "dma")
            for pn in (78, 79):
                gpu.release(pn)
            dma_ctx.release(80)
    finally:
        dma_ctx.close()


def test_10bit_msb_parity(svtme, gpu):
    S = svtme
    w, h = 640, 360
    syn = S.Synth(w, h)
    f10 = {t: syn.frame10(t) for t in (7, 8, 9)}
    for t, f in f10.items():
        gpu.upload(2000 + t, f)
    ctrl = S.derive_controls(6, 35, S.input_resolution_of(w, h), 1)
    job = S.make_job(w, h, ctrl, 2008, (2007,), (2009,), temporal_layer_index=1, ref_count_used=(1, 1),
                     enable_me_8x8=True)
    recs, sbr = gpu.submit(job)
    pyr = {t: S.build_host_pyramid(f, "oracle") for t, f in f10.items()}
    orecs, osbr = S.run_checker(job, pyr[8], {(0, 0): pyr[7], (1, 0): pyr[9]}, "oracle", nthreads=8)
    assert not S.compare_records(orecs, recs, osbr, sbr)
    for t in f10:
        gpu.release(2000 + t)


MCTF_CASES = [  # content, w, h, tf hme_me_level, qp_opt, cur, ref, tl, tf_me_exit_th
    ("pan", 320, 192, 0, 0, 8, 7, 1, 0),
    ("pan", 320, 192, 1, 0, 8, 10, 1, 0),
    ("pan", 640, 360, 2, 1, 8, 9, 0, 9800),
    ("pan", 320, 192, 3, 0, 8, 7, 1, 2600),
    ("noise", 192, 128, 3, 0, 8, 6, 2, 0),
    ("flat", 192, 128, 4, 0, 8, 7, 1, 1),
    ("stripes", 320, 192, 2, 0, 8, 9, 1, 50000),
    # levels 1-2 take k_l1_full: ragged widths and heights (partial 32x32 blocks), fast motion
    # (windows clamped at the picture edges), noise and saturated content (no HME exits)
    ("noise", 200, 136, 2, 1, 8, 7, 1, 0),
    ("vpan", 424, 240, 2, 0, 8, 7, 1, 0),
    ("hpan", 264, 200, 1, 0, 8, 9, 1, 0),
    ("sat", 192, 128, 2, 1, 8, 6, 2, 0),
    ("pan", 72, 40, 1, 0, 8, 7, 1, 0),
    # k_l0_full<4> (HME-L0 quadrants taller than 8 rows) on a last SB row of 8 lines
    # (height 8 mod 64) with whole 16-pixel source dwords: level 1, and level 2 above 480p
    ("pan", 256, 200, 1, 0, 8, 7, 1, 0),
    ("hpan", 1280, 712, 2, 1, 8, 9, 1, 0),
]


@pytest.mark.parametrize("case", MCTF_CASES, ids=lambda c: f"{c[0]}-{c[1]}x{c[2]}-lvl{c[3]}-th{c[8]}")
def test_mctf_parity(svtme, gpu, case):
    """TF-ME jobs (me_type ME_MCTF) on the GPU == the oracle (pinned to the
    reference by tests/golden/tf_cases.json)."""
    S = svtme
    kind, w, h, lvl, qp_opt, cur, ref, tl, th = case
    frames = S.test_frames(kind, w, h, [cur, ref])
    ctrl = S.derive_controls_tf(lvl, qp_opt, 35, S.input_resolution_of(w, h))
    for t, f in frames.items():
        gpu.upload(4000 + t, f)
    job = S.case_job(ctrl, w, h, 4000 + cur, (4000 + ref,), (), tl, me_type=S.ME_MCTF, tf_me_exit_th=th)
    recs, sbr = gpu.submit(job)
    # without per-SB results the split path's records come from the searching
    # wavefronts themselves (direct_records: no k_stage_e launch)
    recs_direct, _ = gpu.submit(job, with_sb_results=False)
    pyr = {t: S.build_host_pyramid(f, "oracle") for t, f in frames.items()}
    ojob = S.case_job(ctrl, w, h, cur, (ref,), (), tl, me_type=S.ME_MCTF, tf_me_exit_th=th)
    orecs, osbr = S.run_checker(ojob, pyr[cur], {(0, 0): pyr[ref]}, "oracle", nthreads=8)
    for t in frames:
        gpu.release(4000 + t)
    errs = S.compare_records(orecs, recs, osbr, sbr)
    assert not errs, errs[:5]
    assert recs_direct.tobytes() == recs.tobytes()


def test_mctf_batch_mixed_outputs(svtme, gpu):
    """A batch of TF-ME jobs (one launch group) where only the middle job asks for
    per-SB results: k_stage_e then runs for every job and rewrites the records the
    direct jobs' wavefronts already wrote. Records equal the single-job ones, with
    and without per-SB results in the batch."""
    import torch

    S = svtme
    w, h = 640, 360
    frames = S.test_frames("pan", w, h, [5, 6, 7, 8, 9])
    for t, f in frames.items():
        gpu.upload(4500 + t, f)
    ctrl = S.derive_controls_tf(2, 1, 35, S.input_resolution_of(w, h))
    jobs = [S.case_job(ctrl, w, h, 4508, (4500 + r,), (), 1, me_type=S.ME_MCTF, tf_me_exit_th=0) for r in (7, 9, 6)]
    single = [gpu.submit(j, with_sb_results=False)[0] for j in jobs]
    nb = single[0].nbytes
    nsb = single[0].shape[0]
    for with_mid_sb in (False, True):
        bufs = [torch.zeros(nb, dtype=torch.uint8, device="cuda") for _ in jobs]
        sbs = [None, torch.zeros(nsb * S.SB_RESULT_DTYPE.itemsize, dtype=torch.uint8, device="cuda"), None]
        torch.cuda.synchronize()  # the zero fills (torch's stream) before the library's streams write
        gpu.submit_batch_device(jobs, [b.data_ptr() for b in bufs],
                                [s.data_ptr() if s is not None else None for s in sbs] if with_mid_sb else None)
        gpu.sync()
        for k, b in enumerate(bufs):
            assert b.cpu().numpy().tobytes() == single[k].tobytes(), (with_mid_sb, k)
    for t in frames:
        gpu.release(4500 + t)


def _controls_case(S, gpu, ctrl, w, h, l0, l1, tl=1, kind="pan"):
    frames = S.test_frames(kind, w, h, sorted(set([8] + list(l0) + list(l1))))
    for t, f in frames.items():
        gpu.upload(5000 + t, f)
    job = S.case_job(ctrl, w, h, 5008, tuple(5000 + t for t in l0), tuple(5000 + t for t in l1), tl)
    recs, sbr = gpu.submit(job)
    pyr = {t: S.build_host_pyramid(f, "oracle") for t, f in frames.items()}
    refs = {(0, i): pyr[t] for i, t in enumerate(l0)}
    refs.update({(1, i): pyr[t] for i, t in enumerate(l1)})
    orecs, osbr = S.run_checker(S.case_job(ctrl, w, h, 8, l0, l1, tl), pyr[8], refs, "oracle", nthreads=8)
    for t in frames:
        gpu.release(5000 + t)
    return S.compare_records(orecs, recs, osbr, sbr)


def test_sr_adjustment_level2_parity(svtme, gpu):
    """enable_me_sr_adjustment == 2 (slot 0's 64x64 SAD resizes the other
    slots' areas, motion_estimation.c:1355-1364): the per-SB full-pel kernel."""
    S = svtme
    ctrl = S.derive_controls(4, 35, S.input_resolution_of(640, 360), 1)
    ctrl.enable_me_sr_adjustment = 2
    assert not _controls_case(S, gpu, ctrl, 640, 360, (7, 6), (9,))


def test_banded_fullpel_parity(svtme, gpu):
    """A fixed 64 x 64 full-pel area (the 1080p bench override): the search
    rows of every (SB, reference) are split over several wavefronts whose
    argmin keys merge with atomic min; run twice to check the keys' reset."""
    S = svtme
    ctrl = S.derive_controls(8, 35, S.input_resolution_of(640, 360), 1)
    ctrl.me_sa.sa_min.width = ctrl.me_sa.sa_min.height = 64
    ctrl.me_sa.sa_max.width = ctrl.me_sa.sa_max.height = 64
    ctrl.me_8x8_var_enabled = 0
    ctrl.enable_me_sr_adjustment = 0
    for _ in range(2):
        assert not _controls_case(S, gpu, ctrl, 640, 360, (7,), ())
    # then a single-band job, then banded again (keys left behind by plain stores)
    assert not _controls_case(S, gpu, S.derive_controls(8, 35, S.input_resolution_of(640, 360), 1), 640, 360,
                              (7, 6), (9, 10))
    assert not _controls_case(S, gpu, ctrl, 640, 360, (7,), ())


@pytest.mark.parametrize("area,th,k32", [((64, 48), "grow", False), ((80, 64), "shrink", False),
                                         ((64, 48), "shrink", True), ((32, 24), "grow", True),
                                         ((48, 32), "shrink", True), ((48, 32), "derived", True)])
def test_banded_fullpel_variance_parity(svtme, gpu, area, th, k32):
    """Banded full-pel search WITH the 8x8-variance centre probe: every band
    re-inserts the probe's key at order 0, which the decode reads as the
    centre; the area grows (x 3/2) or shrinks (/2, /4) after the probe, with
    64-bit and 32-bit argmin keys."""
    S = svtme
    ctrl = S.derive_controls(8, 35, S.input_resolution_of(640, 360), 1)
    ctrl.me_sa.sa_min.width = ctrl.me_sa.sa_max.width = area[0]
    ctrl.me_sa.sa_min.height = ctrl.me_sa.sa_max.height = area[1]
    ctrl.me_8x8_var_enabled = 1
    ctrl.enable_me_sr_adjustment = 0
    ctrl.me_early_exit_th = 0  # check_00_center on as well
    if th == "grow":
        ctrl.me_sr_div4_th, ctrl.me_sr_div2_th, ctrl.me_sr_mult2_th = 0, 0, 0
    elif th == "shrink":
        ctrl.me_sr_div4_th, ctrl.me_sr_div2_th, ctrl.me_sr_mult2_th = 0xFFFFFFF, 0xFFFFFFF, 0xFFFFFFFF
    lib = S.load_product()
    lib.svtme_fp_k32.restype = C.c_bool
    assert lib.svtme_fp_parts(C.byref(ctrl)) > 1, "the case must take the banded path"
    assert lib.svtme_fp_k32(C.byref(ctrl)) == k32
    assert not _controls_case(S, gpu, ctrl, 640, 360, (7, 6), (9,))


@pytest.mark.parametrize("width", [24, 28, 40, 44, 56, 76])
def test_fp_wide_set_split_parity(svtme, gpu, width):
    """k_fp_wide's set loop at area widths that end its 16-position sets in every
    way: whole sets folded two at a time, a lone whole set, and a partial set of
    a whole pair (8 positions), of a whole and a masked pair (12) or none."""
    S = svtme
    ctrl = S.derive_controls(8, 35, S.input_resolution_of(640, 360), 1)
    ctrl.me_sa.sa_min.width = ctrl.me_sa.sa_max.width = width
    ctrl.me_sa.sa_min.height = ctrl.me_sa.sa_max.height = 48
    ctrl.me_8x8_var_enabled = 0
    ctrl.enable_me_sr_adjustment = 0
    lib = S.load_product()
    lib.svtme_fp_wide_lds.restype = C.c_bool
    assert lib.svtme_fp_wide_lds(C.byref(ctrl)), "the case must run k_fp_wide"
    assert not _controls_case(S, gpu, ctrl, 640, 360, (7, 6), (9,))


def test_picture_release_while_read(svtme, gpu):
    """svtme_picture_release does not wait for the device: a job queued before the
    release still reads the released reference (its memory is freed, or reused by
    a picture of the same size, only once that job has run), and a picture that
    reuses released memory holds its own planes."""
    import torch

    S = svtme
    w, h = 640, 360
    syn = S.Synth(w, h)
    cur, ref7, ref9, other = syn.frame(8), syn.frame(7), syn.frame(9), syn.frame(20)
    ctrl = S.derive_controls(8, 35, S.input_resolution_of(w, h), 1)
    for pn, f in ((4208, cur), (4207, ref7), (4209, ref9)):
        gpu.upload(pn, f)
    job = S.make_job(w, h, ctrl, 4208, (4207,), (4209,), temporal_layer_index=1, ref_count_used=(1, 1))
    want = gpu.submit(job)[0]
    n, R = S.sb_total(w, h), S.ref_slots(job)
    bufs = [torch.zeros(n * R * S.REF_RECORD_DTYPE.itemsize, dtype=torch.uint8, device="cuda") for _ in range(3)]
    torch.cuda.synchronize()
    for k, b in enumerate(bufs):  # queued on both lanes, nothing waited for
        gpu.submit_batch_device([job], [b.data_ptr()], lane=k & 1)
    gpu.release(4207)
    gpu.upload_async(4230, other)  # same size: may take the released memory once the jobs have run
    gpu.upload_async(4207, other)  # the released number again, other content
    gpu.sync()
    for b in bufs:
        got = np.frombuffer(b.cpu().numpy().tobytes(), dtype=S.REF_RECORD_DTYPE).reshape(n, R)
        assert not S.compare_records(want, got)
    p_other = S.build_host_pyramid(other, "oracle")
    for pn in (4230, 4207):
        for lv, name in enumerate(("full", "quarter", "sixteenth")):
            assert np.array_equal(gpu.download(pn, lv), getattr(p_other, name)), (pn, name)
    # released and idle now: the next same-size picture reuses memory and holds its own planes
    gpu.release(4230)
    gpu.upload(4231, ref7)
    p7 = S.build_host_pyramid(ref7, "oracle")
    for lv, name in enumerate(("full", "quarter", "sixteenth")):
        assert np.array_equal(gpu.download(4231, lv), getattr(p7, name)), name
    for pn in (4207, 4208, 4209, 4231):
        gpu.release(pn)


def test_picture_upload_async(svtme, gpu):
    """svtme_picture_upload_async: DMA into the resident plane + in-place pyramid
    build on the upload stream; the planes equal the reference's pyramid, a job
    queued before a re-upload of one of its references reads the old planes and
    a job after it the new ones (device outputs, nothing synchronised between),
    and a pinned source behaves like a pageable one."""
    import torch

    S = svtme
    w, h = 328, 200  # not multiples of 64: partial SBs, pad-to-8 columns and rows
    syn = S.Synth(w, h)
    old, new = syn.frame(7), syn.frame(12)
    cur, ref9 = syn.frame(8), syn.frame(9)
    ctrl = S.derive_controls(8, 35, S.input_resolution_of(w, h), 1)
    gpu.upload_async(4108, cur)
    pinned = torch.from_numpy(np.ascontiguousarray(old)).pin_memory()
    gpu.upload_async(4107, pinned.data_ptr(), w, h)
    gpu.upload_async(4109, ref9)
    W8, H8 = (w + 7) & ~7, (h + 7) & ~7
    job = S.make_job(W8, H8, ctrl, 4108, (4107,), (4109,), temporal_layer_index=1, ref_count_used=(1, 1))
    R = S.ref_slots(job)
    n = S.sb_total(W8, H8)
    bufs = [torch.zeros(n * R * S.REF_RECORD_DTYPE.itemsize, dtype=torch.uint8, device="cuda") for _ in range(2)]
    torch.cuda.synchronize()  # the zero fills (torch's stream) before the library's streams write
    gpu.submit_batch_device([job], [bufs[0].data_ptr()])
    gpu.upload_async(4107, new)  # re-upload while the first job may still run
    gpu.submit_batch_device([job], [bufs[1].data_ptr()])
    gpu.sync()
    got = [np.frombuffer(b.cpu().numpy().tobytes(), dtype=S.REF_RECORD_DTYPE).reshape(n, R) for b in bufs]
    p_new = S.build_host_pyramid(new, "oracle")
    for lv, name in enumerate(("full", "quarter", "sixteenth")):
        assert np.array_equal(gpu.download(4107, lv), getattr(p_new, name)), name
        assert np.array_equal(gpu.download(4108, lv), getattr(S.build_host_pyramid(cur, "oracle"), name)), name
    pyr = {8: S.build_host_pyramid(cur, "oracle"), 9: S.build_host_pyramid(ref9, "oracle")}
    for ref7, g in ((S.build_host_pyramid(old, "oracle"), got[0]), (p_new, got[1])):
        orecs, _ = S.run_checker(job, pyr[8], {(0, 0): ref7, (1, 0): pyr[9]}, "oracle", nthreads=8)
        assert not S.compare_records(orecs, g)
    for pn in (4107, 4108, 4109):
        gpu.release(pn)


@pytest.mark.gpu
def test_picture_upload_copy_async_many_threads(svtme, gpu):
    """More concurrent svtme_picture_upload_copy_async callers than staging slots
    (SVTME_UPLOAD_SLOTS = 4): 12 threads upload at once (ctypes drops the GIL in
    the call), every call succeeds -- a caller waits for a free slot instead of
    failing -- and every pyramid equals the reference's."""
    import threading

    S = svtme
    w, h = 328, 200
    syn = S.Synth(w, h)
    ts = list(range(60, 72))
    frames = {t: syn.frame(t) for t in ts}
    errs, go = [], threading.Barrier(len(ts))

    def up(t):
        try:
            go.wait()
            gpu.upload_copy_async(7000 + t, frames[t])
        except Exception as e:  # noqa: BLE001 (reported below)
            errs.append((t, repr(e)))
    th = [threading.Thread(target=up, args=(t,)) for t in ts]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs, errs
    gpu.sync()
    for t in ts:
        p = S.build_host_pyramid(frames[t], "oracle")
        for lv, name in enumerate(("full", "quarter", "sixteenth")):
            assert np.array_equal(gpu.download(7000 + t, lv), getattr(p, name)), (t, name)
        gpu.release(7000 + t)


def test_picture_upload_copy_async_and_pool(svtme, gpu):
    """svtme_picture_upload_copy_async: the rows go through the library's own
    page-locked staging ring (the caller's buffer is never page-locked), so the
    caller may overwrite it as soon as the call returns: more uploads than ring
    slots from ONE reused buffer, each overwritten right after its call, every
    pyramid equal to the reference's; a re-upload waits for the queued job that
    reads the old planes. Pictures come from svtme_reserve_pictures' pool and
    released pictures' memory returns to it (reused, never freed)."""
    import torch

    S = svtme
    w, h = 328, 200
    syn = S.Synth(w, h)
    gpu.reserve_pictures(w, h, 3)
    buf = np.empty((h, w), np.uint8)
    ts = list(range(20, 20 + 2 * 4 + 1))  # > SVTME_UPLOAD_SLOTS uploads from one buffer
    for t in ts:
        buf[:] = syn.frame(t)
        gpu.upload_copy_async(5000 + t, buf)
        buf[:] = 0  # the caller's buffer is free as soon as the call returns
    for t in ts:
        p = S.build_host_pyramid(syn.frame(t), "oracle")
        for lv, name in enumerate(("full", "quarter", "sixteenth")):
            assert np.array_equal(gpu.download(5000 + t, lv), getattr(p, name)), (t, name)
    # a job, then a re-upload of its reference before the job ran (ordering as upload_async)
    ctrl = S.derive_controls(8, 35, S.input_resolution_of(w, h), 1)
    W8, H8 = (w + 7) & ~7, (h + 7) & ~7
    job = S.make_job(W8, H8, ctrl, 5021, (5020,), (5022,), temporal_layer_index=1, ref_count_used=(1, 1))
    R, n = S.ref_slots(job), S.sb_total(W8, H8)
    bufs = [torch.zeros(n * R * S.REF_RECORD_DTYPE.itemsize, dtype=torch.uint8, device="cuda") for _ in range(2)]
    torch.cuda.synchronize()
    gpu.submit_batch_device([job], [bufs[0].data_ptr()])
    buf[:] = syn.frame(40)
    gpu.upload_copy_async(5020, buf)
    gpu.submit_batch_device([job], [bufs[1].data_ptr()])
    gpu.sync()
    got = [np.frombuffer(b.cpu().numpy().tobytes(), dtype=S.REF_RECORD_DTYPE).reshape(n, R) for b in bufs]
    pyr = {t: S.build_host_pyramid(syn.frame(t), "oracle") for t in (20, 21, 22, 40)}
    for ref, g in ((pyr[20], got[0]), (pyr[40], got[1])):
        orecs, _ = S.run_checker(job, pyr[21], {(0, 0): ref, (1, 0): pyr[22]}, "oracle", nthreads=8)
        assert not S.compare_records(orecs, g)
    # released pictures' buffers go back to the pool and serve later uploads
    for t in ts:
        gpu.release(5000 + t)
    gpu.sync()
    for t in ts:
        gpu.upload_copy_async(6000 + t, syn.frame(t))
    for lv, name in enumerate(("full", "quarter", "sixteenth")):
        assert np.array_equal(gpu.download(6000 + ts[-1], lv), getattr(S.build_host_pyramid(syn.frame(ts[-1]), "oracle"), name))
    for t in ts:
        gpu.release(6000 + t)


def test_batched_packed_jobs(svtme, gpu):
    """svtme_submit_pictures_packed_async: several jobs (a TF window's
    (central, reference) pairs) in ONE launch, each with its own ticket and
    host output, equal the same jobs submitted one by one."""
    import ctypes as C

    S = svtme
    w, h = 640, 360
    syn = S.Synth(w, h)
    for t in range(4, 13):
        gpu.upload(7100 + t, syn.frame(t))
    ctrl = S.derive_controls_tf(2, 1, 35, S.input_resolution_of(w, h))
    jobs = [S.case_job(ctrl, w, h, 7108, (7100 + r,), (), 0, me_type=S.ME_MCTF, tf_me_exit_th=0)
            for r in (4, 5, 6, 7, 9, 10, 11, 12)]
    L = S.PackLayout()
    L.n_pus, L.max_cand, L.max_refs, L.full_records, L.sb_results = 0, 0, 0, 1, 0
    exp = [gpu.submit_packed(j, L) for j in jobs]
    n = len(jobs)
    nbytes = len(exp[0])
    ptrs = [gpu.lib.svtme_host_alloc(nbytes) for _ in range(n)]
    arr_jobs = (S.Job * n)(*jobs)
    arr_l = (S.PackLayout * n)(*([L] * n))
    arr_p = (C.c_void_p * n)(*ptrs)
    tickets = (C.c_uint64 * n)()
    gpu.lib.svtme_submit_pictures_packed_async.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(S.Job),
                                                           C.POINTER(S.PackLayout), C.POINTER(C.c_void_p),
                                                           C.POINTER(C.c_uint64)]
    gpu.lib.svtme_submit_pictures_packed_async.restype = C.c_int32
    gpu._check(gpu.lib.svtme_submit_pictures_packed_async(gpu.ctx, 1, n, arr_jobs, arr_l, arr_p, tickets),
               "svtme_submit_pictures_packed_async")
    for k in reversed(range(n)):  # retired in any order
        assert gpu.wait_packed(tickets[k], ptrs[k], nbytes) == exp[k], k
    for t in range(4, 13):
        gpu.release(7100 + t)


def test_lanes_parity(svtme, gpu):
    """svtme_submit_batch_device_lane: batches alternating over the two lanes
    (own streams and scratch, overlapping on the GPU), banded full-pel jobs
    (per-lane argmin keys) and fused jobs in flight together, equal the
    single-lane results; a re-upload of a reference waits for both lanes'
    readers."""
    import torch

    S = svtme
    w, h = 640, 360
    syn = S.Synth(w, h)
    frames = {t: syn.frame(t) for t in (6, 7, 8, 9, 10, 13)}
    for t, f in frames.items():
        gpu.upload(6000 + t, f)
    base = S.derive_controls(8, 35, S.input_resolution_of(w, h), 1)
    band = S.derive_controls(8, 35, S.input_resolution_of(w, h), 1)
    band.me_sa.sa_min.width = band.me_sa.sa_min.height = 64
    band.me_sa.sa_max.width = band.me_sa.sa_max.height = 64
    band.me_8x8_var_enabled = 0
    band.enable_me_sr_adjustment = 0
    jobs = [S.make_job(w, h, base, 6008, (6007, 6006), (6009, 6010), temporal_layer_index=1),
            S.make_job(w, h, band, 6008, (6007,), (), temporal_layer_index=1),
            S.make_job(w, h, base, 6009, (6008, 6007), (6010,), temporal_layer_index=1, ref_count_used=(2, 1))]
    n = S.sb_total(w, h)
    ref = [gpu.submit(j)[0] for j in jobs]  # single lane, synchronous

    def buf(j):
        return torch.zeros(n * S.ref_slots(j) * S.REF_RECORD_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    # every output buffer zero-filled (on torch's stream) before the lanes' jobs write them: the
    # library's streams do not wait for torch's, and a late fill would overwrite a job's records
    outs = [(k, buf(j)) for it in range(6) for k, j in enumerate(jobs)]
    after = buf(jobs[0])
    torch.cuda.synchronize()
    for i, (k, b) in enumerate(outs):
        gpu.submit_batch_device([jobs[k]], [b.data_ptr()], lane=(i // len(jobs) + k) & 1)
    # re-upload ref 6007 asynchronously while both lanes may still read it, then search again
    gpu.upload_async(6007, frames[13])
    gpu.submit_batch_device([jobs[0]], [after.data_ptr()], lane=1)
    gpu.sync()
    for k, b in outs:
        got = np.frombuffer(b.cpu().numpy().tobytes(), dtype=S.REF_RECORD_DTYPE).reshape(n, -1)
        assert not S.compare_records(ref[k], got), k
    gpu.upload(6007, frames[13])
    want = gpu.submit(jobs[0])[0]
    got = np.frombuffer(after.cpu().numpy().tobytes(), dtype=S.REF_RECORD_DTYPE).reshape(n, -1)
    assert not S.compare_records(want, got)
    assert S.compare_records(ref[0], got)  # the new reference changed the result
    for t in frames:
        gpu.release(6000 + t)


def test_picture_invalidate(svtme, gpu):
    """svtme_picture_invalidate (TF re-decimation, temporal_filtering.c:3895-3931):
    the resident pyramid is rebuilt from the new planes, jobs queued before it
    read the old planes, jobs after it the new ones; a non-resident picture is
    refused."""
    S = svtme
    w, h = 320, 192
    syn = S.Synth(w, h)
    old, new = syn.frame(7), syn.frame(11)
    cur, ref9 = syn.frame(8), syn.frame(9)
    ctrl = S.derive_controls(8, 35, S.input_resolution_of(w, h), 1)
    for pn, f in ((3008, cur), (3007, old), (3009, ref9)):
        gpu.upload(pn, f)
    job = S.make_job(w, h, ctrl, 3008, (3007,), (3009,), temporal_layer_index=1, ref_count_used=(1, 1))
    before = gpu.submit(job)
    gpu.invalidate(3007, new)
    after = gpu.submit(job)
    p_new = S.build_host_pyramid(new, "oracle")
    for lv, name in enumerate(("full", "quarter", "sixteenth")):
        assert np.array_equal(gpu.download(3007, lv), getattr(p_new, name)), name
    pyr = {8: S.build_host_pyramid(cur, "oracle"), 9: S.build_host_pyramid(ref9, "oracle")}
    for ref7, got in ((S.build_host_pyramid(old, "oracle"), before), (p_new, after)):
        orecs, osbr = S.run_checker(job, pyr[8], {(0, 0): ref7, (1, 0): pyr[9]}, "oracle", nthreads=8)
        assert not S.compare_records(orecs, got[0], osbr, got[1])
    assert not S.compare_records(before[0], after[0]) == []  # the new planes changed the result
    with pytest.raises(RuntimeError):
        gpu.invalidate(123456, new)
    for pn in (3007, 3008, 3009):
        gpu.release(pn)


with open(os.path.join(GOLD, "me_cases.json")) as _fh:
    GOLD_ME_CASES = json.load(_fh)


@pytest.mark.parametrize("case", GOLD_ME_CASES, ids=lambda c: c["name"])
def test_picture_vs_reference_golden(svtme, gpu, case):
    """The GPU job against the reference's own outputs (tests/golden/me_*.npz,
    made by libsvtref from the reference sources), controls as stored with the
    case: the derived controls and the real-time tune's reduce_hme_l0_sr_th
    cases (HME-L0 areas of slots 1-7 from slot 0's centre)."""
    S = svtme
    ctrl = S.Controls.from_dict(case["ctrl"])
    w, h, l0, l1 = case["w"], case["h"], tuple(case["l0"]), tuple(case["l1"])
    frames = S.test_frames(case["content"], w, h, sorted(set([8] + list(l0) + list(l1))))
    job = S.case_job(ctrl, w, h, 8, l0, l1, case["tl"], **case["extra"])
    for t, f in frames.items():
        gpu.upload(3000 + t, f)
    job.picture_number = 3000 + 8
    for i, t in enumerate(l0):
        job.ref_picture_number[0][i] = 3000 + t
    for i, t in enumerate(l1):
        job.ref_picture_number[1][i] = 3000 + t
    try:
        recs, sbr = gpu.submit(job)
    finally:
        for t in frames:
            gpu.release(3000 + t)
    z = np.load(os.path.join(GOLD, f"me_{case['name']}.npz"))
    exp_recs = z["records"].view(S.REF_RECORD_DTYPE).reshape(recs.shape)
    exp_sb = z["sb"].view(S.SB_RESULT_DTYPE).reshape(sbr.shape)
    errs = S.compare_records(exp_recs, recs, exp_sb, sbr)
    assert not errs, errs[:5]
    assert S.records_checksum(recs, sbr) == case["checksum"]


@pytest.mark.parametrize("case", [c for c in GOLD_ME_CASES if "_rt" in c["name"]], ids=lambda c: c["name"])
def test_realtime_split_path_vs_reference_golden(svtme, gpu, case):
    """The real-time tune's HME-L0 reduction on the split HME path (k_stage_a ->
    k_stage_d<true> -> k_stage_a<true> -> k_stage_d), forced for widths k_hme
    would take (svtme_set_paths), against the reference's outputs."""
    gpu.set_paths(svtme.PATH_NO_FUSED_HME)
    try:
        test_picture_vs_reference_golden(svtme, gpu, case)
    finally:
        gpu.set_paths(0)


def test_job_validation_errors(svtme, gpu):
    """Malformed jobs are refused with SVTME_ERR_BAD_PARAMETER and a message,
    before anything is launched, and the context stays usable: a picture that is
    not resident, a size that is not a multiple of 8 or does not match the
    resident planes, an SB range outside the picture, reference counts beyond
    the reference's 2 x 4, an unknown me_type."""
    import copy

    S = svtme
    w, h = 320, 192
    syn = S.Synth(w, h)
    frames = {t: syn.frame(t) for t in (7, 8)}
    for t, f in frames.items():
        gpu.upload(6000 + t, f)
    ctrl = S.derive_controls(8, 35, S.input_resolution_of(w, h), 1)
    good = S.make_job(w, h, ctrl, 6008, (6007,), (), temporal_layer_index=1, ref_count_used=(1, 0))
    ok_recs, _ = gpu.submit(good)

    def bad(mut, needle):
        j = copy.copy(good)
        mut(j)
        with pytest.raises(RuntimeError) as ei:
            gpu.submit(j)
        assert "0x" in str(ei.value) and needle in str(ei.value), str(ei.value)

    bad(lambda j: setattr(j, "picture_number", 6999), "not resident")
    bad(lambda j: j.ref_picture_number[0].__setitem__(0, 6998), "not resident")
    bad(lambda j: setattr(j, "width", w + 4), "multiple of 8")
    bad(lambda j: setattr(j, "width", w - 64), "is 320x192")
    bad(lambda j: setattr(j, "sb_begin", S.sb_total(w, h)), "outside the picture")
    bad(lambda j: setattr(j, "sb_count", S.sb_total(w, h) + 1), "outside the picture")
    bad(lambda j: j.num_refs.__setitem__(0, 5), "reference counts")
    bad(lambda j: setattr(j, "me_type", 7), "me_type")
    # the context still serves a good job with the same result
    again, _ = gpu.submit(good)
    assert again.tobytes() == ok_recs.tobytes()
    for t in frames:
        gpu.release(6000 + t)
