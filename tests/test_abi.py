"""CPU: the drop-in boundary (include/svtme.h) — the C-ABI library loads, exports
every declared entry point, and the header's struct layouts agree with the
Python/numpy mirrors used by the host code and the tests. No GPU calls here.
"""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import PKG, ROOT

HEADER = os.path.join(ROOT, "include", "svtme.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"^static inline[^\n]*", "", text, flags=re.M)  # header-only helpers (svtme_packed_sb_bytes)
    names = set(re.findall(r"^\s*[A-Za-z_][\w \*]*?\b(svt\w+)\s*\(", text, flags=re.M))
    return sorted(names)


def test_header_declares_the_interfaces():
    names = declared_functions()
    # job API + every rtcd variant the header promises
    for n in ("svtme_ctx_create", "svtme_submit_picture", "svtme_submit_picture_device", "svtme_derive_controls",
              "svt_sad_loop_kernel_hip", "svt_nxm_sad_kernel_hip", "svt_aom_downsample_2d_hip",
              "svt_ext_all_sad_calculation_8x8_16x16_hip", "svt_aom_sad_16b_kernel_hip"):
        assert n in names, n


def test_library_exports_every_declared_function():
    lib = C.CDLL(os.path.join(PKG, "libsvtme.so"))
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


PROBE = r"""
#include <stddef.h>
#include <stdio.h>
#include "svtme.h"
#define P(T) printf(#T " %zu\n", sizeof(T))
#define O(T, f) printf(#T "." #f " %zu\n", offsetof(T, f))
int main(void) {
    P(svtme_controls); P(svtme_job); P(svtme_ref_record); P(svtme_sb_result);
    O(svtme_job, ctrl); O(svtme_job, sb_begin); O(svtme_job, sb_count); O(svtme_job, ref_picture_number);
    O(svtme_ref_record, best_mv); O(svtme_ref_record, hme_sad); O(svtme_ref_record, hme_sc_x);
    O(svtme_ref_record, zz_sad); O(svtme_ref_record, searched); O(svtme_ref_record, do_ref);
    O(svtme_ref_record, tf_early_exit); O(svtme_job, me_type); O(svtme_job, tf_me_exit_th);
    O(svtme_sb_result, me_candidate_array); O(svtme_sb_result, me_mv_array); O(svtme_sb_result, me_distortion);
    O(svtme_sb_result, me_8x8_cost_variance); O(svtme_sb_result, rc_me_allow_gm);
    O(svtme_controls, prehme_sa_cfg); O(svtme_controls, me_early_exit_th);
    O(svtme_controls, prev_me_stage_based_exit_th);
    printf("SVTME_MAX_TICKETS %d\n", SVTME_MAX_TICKETS);
    return 0;
}
"""


def test_struct_layouts_match_mirrors(svtme, tmp_path):
    S = svtme
    src = tmp_path / "probe.c"
    src.write_text(PROBE)
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                                check=True).stdout.split("\n") if line)
    got = {k: int(v) for k, v in got.items()}
    assert got["SVTME_MAX_TICKETS"] == S.MAX_TICKETS
    assert got["svtme_controls"] == C.sizeof(S.Controls)
    assert got["svtme_job"] == C.sizeof(S.Job)
    assert got["svtme_ref_record"] == S.REF_RECORD_DTYPE.itemsize == 704
    assert got["svtme_sb_result"] == S.SB_RESULT_DTYPE.itemsize
    assert got["svtme_job.ctrl"] == S.Job.ctrl.offset
    assert got["svtme_job.sb_begin"] == S.Job.sb_begin.offset
    assert got["svtme_job.sb_count"] == S.Job.sb_count.offset
    assert got["svtme_job.ref_picture_number"] == S.Job.ref_picture_number.offset
    assert got["svtme_job.me_type"] == S.Job.me_type.offset
    assert got["svtme_job.tf_me_exit_th"] == S.Job.tf_me_exit_th.offset
    for f in ("best_mv", "hme_sad", "hme_sc_x", "zz_sad", "searched", "do_ref", "tf_early_exit"):
        assert got[f"svtme_ref_record.{f}"] == S.REF_RECORD_DTYPE.fields[f][1], f
    for f in ("me_candidate_array", "me_mv_array", "me_distortion", "me_8x8_cost_variance", "rc_me_allow_gm"):
        assert got[f"svtme_sb_result.{f}"] == S.SB_RESULT_DTYPE.fields[f][1], f
    for f in ("prehme_sa_cfg", "me_early_exit_th", "prev_me_stage_based_exit_th"):
        assert got[f"svtme_controls.{f}"] == getattr(S.Controls, f).offset, f


def test_host_geometry_helpers(svtme):
    """svtme_sb_total / svtme_job_ref_slots (host code in libsvtme.so) vs the mirrors."""
    S = svtme
    lib = S.load_product()
    for w, h in ((64, 64), (65, 64), (3840, 2160), (1920, 1080), (136, 8), (7680, 4320)):
        assert lib.svtme_sb_total(w, h) == S.sb_total(w, h) == ((w + 63) // 64) * ((h + 63) // 64)
    ctrl = S.Controls()
    for l0, l1 in (((7,), ()), ((7, 6), (9,)), ((7, 6, 5, 4), (9, 10, 11))):
        job = S.make_job(320, 192, ctrl, 8, l0, l1)
        assert lib.svtme_job_ref_slots(C.byref(job)) == S.ref_slots(job) == len(l0) + len(l1)


def test_product_fails_loudly_without_a_device(svtme):
    """No CPU fallback: without a usable GPU the product refuses (status + message)."""
    S = svtme
    lib = S.load_product()
    try:
        import torch

        if torch.cuda.is_available():
            pytest.skip("a GPU is present")
    except ImportError:
        pass
    ctx = C.c_void_p()
    st = lib.svtme_ctx_create(0, C.byref(ctx))
    assert st != 0
    assert lib.svtme_last_error()
