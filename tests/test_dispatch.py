"""Host-side kernel dispatch of the full-pel stage (no GPU needed: pure host
functions of libsvtme.so). The 64x64 override (BASELINE configs[1]) takes
k_fp_wide (svtme_stages.hip) with bands in groups of 4 of at most 8 rows; no
default preset's controls change path."""
import ctypes as C
import math

import pytest


@pytest.fixture(scope="module")
def lib(svtme):
    lib = svtme.load_product()
    for f in ("svtme_fp_wide_lds", "svtme_fp_wide", "svtme_fp_k32"):
        getattr(lib, f).argtypes = [C.POINTER(svtme.Controls)]
        getattr(lib, f).restype = C.c_bool
    lib.svtme_fp_parts.argtypes = [C.POINTER(svtme.Controls)]
    lib.svtme_fp_parts.restype = C.c_uint32
    return lib


def test_override_takes_k_fp_wide(svtme, lib):
    import workloads as W

    job = W.workload_job("1080p_sa64")
    c = job.ctrl
    assert lib.svtme_fp_wide_lds(C.byref(c))
    parts = lib.svtme_fp_parts(C.byref(c))
    h = c.me_sa.sa_max.height
    assert parts % 4 == 0 and parts >= math.ceil(h / 8) and parts <= 16
    # LDS rows of a workgroup: 4 bands + 62 (FPW_ROWS = 96)
    assert 4 * math.ceil(h / parts) + 62 <= 96


def test_no_default_preset_changes_path(svtme, lib):
    for m in range(14):
        for res in range(7):
            for tl in range(4):
                c = svtme.derive_controls(m, 35, res, tl)
                assert not lib.svtme_fp_wide_lds(C.byref(c)), (m, res, tl)
    for lvl in range(5):
        for res in range(7):
            c = svtme.derive_controls_tf(lvl, 0, 35, res)
            assert not lib.svtme_fp_wide_lds(C.byref(c)), (lvl, res)


def test_full_sad_and_64bit_keys_keep_the_register_path(svtme, lib):
    import workloads as W

    c = W.workload_job("1080p_sa64").ctrl
    c.me_search_method = svtme.FULL_SAD_SEARCH
    assert not lib.svtme_fp_wide_lds(C.byref(c))
    c = W.workload_job("1080p_sa64").ctrl
    c.me_sa.sa_max.width = c.me_sa.sa_min.width = 96  # wider than the LDS row
    assert not lib.svtme_fp_wide_lds(C.byref(c))
