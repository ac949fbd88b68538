"""CPU parity of the checker and of the product's host logic.

The oracle (oracle/svtme_oracle.c -> liboracle.so) is a from-scratch C
restatement of the reference's open-loop ME; it is the checker every GPU
parity test compares against. Here it is pinned:

* against the golden vectors in tests/golden/ (expected records / SB results
  produced by the reference's own motion_estimation.c compiled from source,
  C and AVX2 kernels agreeing; see tests/golden/make_golden.py), bit-exact;
* against the reference library itself (oracle/_ref/libsvtref.so) on further
  inputs when that library is present (build container only);
* the product's C++ restatement of svt_aom_sig_deriv_me
  (svtme_derive_controls in libsvtme.so, host code) against the reference's
  outputs over presets x resolutions x layers x QPs.
"""
import json
import os

import numpy as np
import pytest

from conftest import ROOT, ref_available

GOLD = os.path.join(ROOT, "tests", "golden")


def _golden_controls():
    with open(os.path.join(GOLD, "controls.json")) as fh:
        return json.load(fh)


with open(os.path.join(GOLD, "me_cases.json")) as _fh:
    ME_CASES = json.load(_fh)


@pytest.mark.parametrize("case", ME_CASES, ids=lambda c: c["name"])
def test_oracle_vs_golden(svtme, case):
    S = svtme
    ctrl = S.Controls.from_dict(case["ctrl"])
    recs, sbr = S.run_case_checker(case["content"], case["w"], case["h"], ctrl, 8, tuple(case["l0"]),
                                   tuple(case["l1"]), case["tl"], checker="oracle", nthreads=4, **case["extra"])
    z = np.load(os.path.join(GOLD, f"me_{case['name']}.npz"))
    exp_recs = z["records"].view(S.REF_RECORD_DTYPE).reshape(recs.shape)
    exp_sb = z["sb"].view(S.SB_RESULT_DTYPE).reshape(sbr.shape)
    errs = S.compare_records(exp_recs, recs, exp_sb, sbr)
    assert not errs, errs[:5]
    assert S.records_checksum(recs, sbr) == case["checksum"]


@pytest.mark.parametrize("case", ME_CASES[:4], ids=lambda c: c["name"])
def test_oracle_pyramid_vs_golden(svtme, case):
    import hashlib

    S = svtme
    f = S.test_frames(case["content"], case["w"], case["h"], [8])[8]
    p = S.build_host_pyramid(f, "oracle")
    for k, d in case["pyramid_sha256"].items():
        assert hashlib.sha256(np.ascontiguousarray(getattr(p, k)).tobytes()).hexdigest() == d, k


def test_product_derive_controls_vs_golden(svtme):
    """svtme_derive_controls (product host code) == svt_aom_sig_deriv_me."""
    S = svtme
    gold = _golden_controls()
    bad = []
    for m, qp, res, tl, idx in gold["rows"]:
        got = json.loads(json.dumps(S.derive_controls(m, qp, res, tl).as_dict()))
        if got != gold["unique"][idx]:
            diff = {k: (got.get(k), v) for k, v in gold["unique"][idx].items() if got.get(k) != v}
            bad.append(((m, qp, res, tl), diff))
    assert not bad, bad[:3]


@pytest.mark.skipif(not ref_available(), reason="oracle/_ref not built (needs /root/reference)")
@pytest.mark.parametrize("preset,tl,size,kind", [
    (2, 1, (200, 120), "pan"), (5, 0, (480, 272), "pan"), (7, 2, (320, 184), "noise"),
    (10, 1, (256, 144), "stripes"), (13, 3, (320, 192), "pan"), (6, 1, (96, 56), "sat"),
])
def test_oracle_vs_ref(svtme, preset, tl, size, kind):
    S = svtme
    w, h = size
    ctrl = S.ref_derive_controls(preset, 35, S.input_resolution_of(w, h), tl)
    l0, l1 = (7, 6), (9,)
    a = S.run_case_checker(kind, w, h, ctrl, 8, l0, l1, tl, checker="oracle", nthreads=4)
    S.load_ref().svtref_set_simd(1)
    b = S.run_case_checker(kind, w, h, ctrl, 8, l0, l1, tl, checker="ref", nthreads=4)
    errs = S.compare_records(b[0], a[0], b[1], a[1])
    assert not errs, errs[:5]


# ---------------------------------------------------------------------------
# TF-ME (me_type ME_MCTF, temporal_filtering.c:3127-3174): same path, other
# controls (svt_aom_sig_deriv_me_tf) and flow (no pruning, undistanced full-pel
# area, HME-only exit, no candidates)
# ---------------------------------------------------------------------------
with open(os.path.join(GOLD, "tf_cases.json")) as _fh:
    TF_CASES = json.load(_fh)


@pytest.mark.parametrize("case", TF_CASES, ids=lambda c: c["name"])
def test_oracle_tf_vs_golden(svtme, case):
    S = svtme
    ctrl = S.Controls.from_dict(case["ctrl"])
    recs, sbr = S.run_case_checker(case["content"], case["w"], case["h"], ctrl, case["cur"], tuple(case["l0"]), (),
                                   case["tl"], checker="oracle", nthreads=4, **case["extra"])
    z = np.load(os.path.join(GOLD, f"me_{case['name']}.npz"))
    exp_recs = z["records"].view(S.REF_RECORD_DTYPE).reshape(recs.shape)
    exp_sb = z["sb"].view(S.SB_RESULT_DTYPE).reshape(sbr.shape)
    errs = S.compare_records(exp_recs, recs, exp_sb, sbr)
    assert not errs, errs[:5]
    assert int(recs["tf_early_exit"].sum()) == case["tf_exits"]
    assert S.records_checksum(recs, sbr) == case["checksum"]


def test_product_derive_controls_tf_vs_golden(svtme):
    """svtme_derive_controls_tf (product host code) == svt_aom_sig_deriv_me_tf."""
    S = svtme
    with open(os.path.join(GOLD, "controls_tf.json")) as fh:
        gold = json.load(fh)
    bad = []
    for lvl, qp_opt, qp, res, idx in gold["rows"]:
        got = json.loads(json.dumps(S.derive_controls_tf(lvl, qp_opt, qp, res).as_dict()))
        if got != gold["unique"][idx]:
            diff = {k: (got.get(k), v) for k, v in gold["unique"][idx].items() if got.get(k) != v}
            bad.append(((lvl, qp_opt, qp, res), diff))
    assert not bad, bad[:3]


@pytest.mark.skipif(not ref_available(), reason="oracle/_ref not built (needs /root/reference)")
@pytest.mark.parametrize("lvl,th,kind", [(0, 0, "pan"), (2, 30000, "noise"), (4, 3000, "pan")])
def test_oracle_tf_vs_ref(svtme, lvl, th, kind):
    S = svtme
    w, h = 256, 144
    ctrl = S.ref_derive_controls_tf(lvl, 1, 35, S.input_resolution_of(w, h))
    kw = dict(me_type=S.ME_MCTF, tf_me_exit_th=th)
    a = S.run_case_checker(kind, w, h, ctrl, 8, (6,), (), 1, checker="oracle", nthreads=4, **kw)
    S.load_ref().svtref_set_simd(1)
    b = S.run_case_checker(kind, w, h, ctrl, 8, (6,), (), 1, checker="ref", nthreads=4, **kw)
    errs = S.compare_records(b[0], a[0], b[1], a[1])
    assert not errs, errs[:5]
