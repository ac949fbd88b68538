"""GPU parity of the wide full-pel stage k_fp_wide (svtme_stages.hip) against
the CPU oracle, bit-exact: the 64x64 full-pel area of BASELINE configs[1] and
a 40x40 area with the 8x8-variance probe and resize (areas 16 .. 64 wide),
on picture sizes whose SBs take the fused k_hme (width a multiple of 64) and
the split HME path (ragged width), with content that drives the zz early exit
(1x1 areas: the masked last pair), ties (flat, stripes) and the pan."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def controls(S, area: int, var: bool):
    c = S.derive_controls(8, 35, S.input_resolution_of(1920, 1080), 1)
    c.me_sa.sa_min.width = c.me_sa.sa_min.height = area
    c.me_sa.sa_max.width = c.me_sa.sa_max.height = area
    c.enable_me_sr_adjustment = 0
    if not var:
        c.me_8x8_var_enabled = 0
    else:  # thresholds that resize most areas up or down
        c.me_8x8_var_enabled = 1
        c.me_sr_mult2_th, c.me_sr_div2_th, c.me_sr_div4_th = 60000, 4000, 1500
    return c


CASES = [
    # content, w, h, area, var, l0, l1
    ("pan", 320, 192, 64, False, (7,), ()),
    ("pan", 320, 192, 64, False, (7, 6), (9,)),
    ("noise", 256, 128, 64, False, (7,), (9,)),
    ("flat", 256, 128, 64, False, (7,), ()),
    ("stripes", 320, 192, 64, False, (7, 6), ()),
    ("pan", 200, 136, 64, False, (7,), (9,)),
    ("pan", 72, 40, 64, False, (7,), ()),
    ("pan", 320, 192, 40, True, (7, 6), (9,)),
    ("noise", 256, 128, 40, True, (7,), ()),
    ("stripes", 200, 136, 40, True, (7,), (9,)),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0]}-{c[1]}x{c[2]}-sa{c[3]}{'-var' if c[4] else ''}-{len(c[5])}+{len(c[6])}")
def test_fp_wide_vs_oracle(svtme, gpu, case):
    S = svtme
    kind, w, h, area, var, l0, l1 = case
    ctrl = controls(S, area, var)
    lib = S.load_product()
    lib.svtme_fp_wide_lds.argtypes = [C.POINTER(S.Controls)]
    lib.svtme_fp_wide_lds.restype = C.c_bool
    assert lib.svtme_fp_wide_lds(C.byref(ctrl))  # the case exercises k_fp_wide
    frames = S.test_frames(kind, w, h, sorted(set([8] + list(l0) + list(l1))))
    res = S.input_resolution_of(w, h)
    mk = dict(temporal_layer_index=1, enable_me_8x8=(res <= S.RES_720P), ref_count_used=(max(len(l0), 1), len(l1)))
    job = S.make_job(w, h, ctrl, 8, l0, l1, **mk)
    for t, f in frames.items():
        gpu.upload(4000 + t, f)
    job.picture_number = 4008
    for i, t in enumerate(l0):
        job.ref_picture_number[0][i] = 4000 + t
    for i, t in enumerate(l1):
        job.ref_picture_number[1][i] = 4000 + t
    try:
        recs, sbr = gpu.submit(job)
    finally:
        for t in frames:
            gpu.release(4000 + t)
    pyr = {t: S.build_host_pyramid(f, "oracle") for t, f in frames.items()}
    refs = {(0, i): pyr[t] for i, t in enumerate(l0)}
    refs.update({(1, i): pyr[t] for i, t in enumerate(l1)})
    orecs, osbr = S.run_checker(S.make_job(w, h, ctrl, 8, l0, l1, **mk), pyr[8], refs, "oracle", nthreads=8)
    errs = S.compare_records(orecs, recs, osbr, sbr)
    assert not errs, errs[:5]
    assert np.array_equal(orecs.view(np.uint8), recs.view(np.uint8))
