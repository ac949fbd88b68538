"""CPU: the encoder-side binding (integration/svtme_svt_glue.c) compiles against
the reference's own headers (/root/reference/Source, build container only):
the rtcd registration assigns the exact pointer names of aom_dsp_rtcd.h, the
controls / job / scatter code reads and writes real MeContext,
PictureParentControlSet and MeSbResults fields. Compiled with gcc -c (not run:
it needs the whole encoder around it)."""
import os
import subprocess

import pytest

from conftest import ROOT

REF = "/root/reference/Source"
GLUE = os.path.join(ROOT, "integration", "svtme_svt_glue.c")


def _incs():
    return [f"-I{REF}/API", f"-I{REF}/Lib/Codec", f"-I{REF}/Lib/C_DEFAULT", f"-I{REF}/Lib/Globals",
            f"-I{os.path.dirname(REF)}/third_party/aom_dsp/inc", f"-I{os.path.dirname(REF)}/third_party",
            f"-I{ROOT}/include"]


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference headers only in the build container")
def test_glue_compiles_against_reference_headers(tmp_path):
    obj = str(tmp_path / "glue.o")
    r = subprocess.run(["gcc", "-std=gnu11", "-Wall", "-Werror", "-Wno-unused-function", "-DARCH_X86_64=1",
                        "-DEN_AVX512_SUPPORT=0", "-c", "-o", obj, GLUE] + _incs(), capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    syms = subprocess.run(["nm", obj], capture_output=True, text=True).stdout
    # defines the glue, binds the reference's rtcd pointers and the library's C ABI
    for s in ("T svt_aom_setup_rtcd_hip_parity", "T svtme_controls_from_me_context", "T svtme_job_from_pcs",
              "T svtme_job_from_tf", "T svtme_scatter_sb", "T svtme_motion_estimation_b64", "T svtme_picture_changed",
              "U svt_sad_loop_kernel_hip", "U svt_pme_sad_loop_kernel_hip", "U svtme_rtcd_failed",
              "U svtme_submit_pictures_packed_async", "U svtme_ticket_wait_timed", "U svtme_picture_upload_async",
              "U svtme_picture_upload_copy_async", "U svtme_reserve_pictures",
              "U svtme_picture_release", "U svt_aom_motion_estimation_b64"):
        assert s in syms, s
    for ptr in ("svt_sad_loop_kernel", "svt_nxm_sad_kernel", "downsample_2d", "sad_16b_kernel",
                "svt_ext_all_sad_calculation_8x8_16x16", "svt_ext_eight_sad_calculation_32x32_64x64",
                "svt_initialize_buffer_32bits", "svt_ext_sad_calculation_8x8_16x16",
                "svt_ext_sad_calculation_32x32_64x64", "svt_pme_sad_loop_kernel"):
        assert f" {ptr}\n" in syms, ptr  # the RTCD_EXTERN pointer itself (aom_dsp_rtcd.h)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference headers only in the build container")
def test_glue_wrap_build_exports_wrappers(tmp_path):
    """-DSVTME_GLUE_WRAP (the --wrap link of oracle/encoder.mk) defines the
    wrappers (the SB function, re-decimation, each encoder's init and deinit, the
    end of each picture's analysis) and calls through to the encoder's own
    functions."""
    obj = str(tmp_path / "glue_wrap.o")
    r = subprocess.run(["gcc", "-std=gnu11", "-Wall", "-Werror", "-DSVTME_GLUE_WRAP", "-DARCH_X86_64=1",
                        "-DEN_AVX512_SUPPORT=0", "-c", "-o", obj, GLUE] + _incs(), capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    syms = subprocess.run(["nm", obj], capture_output=True, text=True).stdout
    for s in ("T __wrap_svt_aom_motion_estimation_b64", "T __wrap_svt_aom_downsample_filtering_input_picture",
              "U __real_svt_aom_motion_estimation_b64", "U __real_svt_aom_downsample_filtering_input_picture",
              "T __wrap_svt_av1_enc_deinit", "U __real_svt_av1_enc_deinit",
              "T __wrap_svt_av1_enc_init", "U __real_svt_av1_enc_init",
              "T __wrap_svt_post_full_object", "U __real_svt_post_full_object"):
        assert s in syms, s


def test_integration_doc_names_real_pointers():
    """INTEGRATION.md's registration example uses the reference's pointer names."""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    assert "svt_aom_downsample_2d  " not in text and "svt_aom_sad_16b_kernel  " not in text
    assert "downsample_2d" in text and "sad_16b_kernel" in text
