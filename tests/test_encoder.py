"""End-to-end: the reference encoder's bitstream is byte-identical with this
library's ME in place of its own (the reference's CI
checks its encoder the same way, .gitlab/workflows/linux/.gitlab-ci.yml:354-370).

CPU: svtav1enc_ora -- integration/svtme_svt_glue.c over the oracle-backed job
API -- against the unmodified encoder; pins every field the glue reads from
and writes into the encoder (PA-ME and TF-ME, GM inputs, candidate arrays),
the upload / re-decimation ordering and the pyramid (SVTME_GLUE_VERIFY compares
every uploaded pyramid with the encoder's own planes).
GPU: svtav1enc_gpu -- the same glue over libsvtme.so on the MI355X.
The encoders are built in the build container by oracle/encoder.mk from the
reference's sources; without them the tests skip.
"""
import os

import pytest

import encoder_harness as E

CPU_CASES = ["ra360_p12", "240p_p8_ragged", "360p_p4", "360p_p8_notf", "360p_superres", "1080p_p8", "4k_p8",
             "360p_p8_lowdelay", "360p_p10_lowdelay", "240p_p8_lowdelay", "360p_p8_2pass", "360p_p8_2ch"]
GPU_CASES = [c for c in E.CASES if c != "4k_p8_64f"]  # the 64-frame encode is scripts/glue_rate.py's


@pytest.fixture(scope="module")
def workdir(tmp_path_factory):
    return str(tmp_path_factory.mktemp("enc"))


@pytest.mark.skipif(not (E.available("ref") and E.available("ora")), reason="encoders built by oracle/encoder.mk")
@pytest.mark.parametrize("case", CPU_CASES)
def test_bitstream_identical_oracle_backend(case, workdir):
    r = E.check(case, "ora", workdir)
    assert r["sbs"] > 0 and r["fallback_sbs"] == 0
    assert r["verified_planes"] == 3 * r["uploads"]
    assert r["verified_job_planes"] >= 3 * (r["pa_jobs"] + r["tf_jobs"])
    assert r["eager_uploads"] > 0
    _no_rtcd_registered(r)


@pytest.mark.skipif(not (E.available("ref") and E.available("ora")), reason="encoders built by oracle/encoder.mk")
@pytest.mark.parametrize("case", ["360p_p8_2pass", "360p_p8_2ch"])
def test_two_encoders_in_one_process(case, workdir):
    """Two encoders in one process -- the passes of a 2-pass encode one after the
    other, two --nch channels at once with different content at the same picture
    numbers -- each keep their own resident pictures (a picture-number range per
    encoder): both bitstreams equal the reference's, every job's pictures equal
    the encoder's planes (SVTME_GLUE_VERIFY), and each teardown releases its
    encoder's pictures."""
    r = E.check(case, "ora", workdir)
    assert r["encoders"] == 2 and r["released_at_teardown"] > 0 and r["fallback_sbs"] == 0
    assert r["verified_job_planes"] >= 3 * (r["pa_jobs"] + r["tf_jobs"])


@pytest.mark.skipif(not (E.available("ref") and E.available("ora")), reason="encoders built by oracle/encoder.mk")
def test_encoder_beyond_slot_cap(workdir):
    """More live encoders than the glue has slots (SVTME_GLUE_MAX_ENC=1 lowers the
    cap of GLUE_MAX_ENC for the test): the second channel gets no slot, so it runs
    the encoder's own ME for every SB and its pictures never become resident --
    none pinned, uploaded or marked stale under the first encoder's picture
    numbers (its re-decimations used to alias slot 0's namespace). Both
    bitstreams equal the reference's, the first encoder's every job passes
    SVTME_GLUE_VERIFY, and only the second's SBs fall back."""
    case = "360p_p8_2ch"
    ref = E.encode("ref", case, workdir)
    one = E.encode("ora", case, workdir, {"SVTME_GLUE_MAX_ENC": "1"})
    g = one["glue"]
    assert one["md5"] == ref["md5"]
    assert g["encoders"] == 1 and g["sbs"] > 0 and g["fallback_sbs"] > 0, g
    assert g["verified_job_planes"] >= 3 * (g["pa_jobs"] + g["tf_jobs"]), g


@pytest.mark.skipif(not (E.available("ref") and E.available("ora")), reason="encoders built by oracle/encoder.mk")
@pytest.mark.parametrize("case", ["ra360_p12", "360p_p8_lowdelay", "240p_p8_ragged", "360p_p4"])
def test_jobs_prefetched_at_picture_decision(case, workdir):
    """Every PA-ME job is submitted when picture decision posts the picture's ME
    tasks (pd_process.c:3544-3556), and every TF-ME pair of a window when it
    posts the window's filtering tasks (:3404-3426), built from the encoder's
    own svt_aom_sig_deriv_me[_tf] into a scratch context: the ME threads' SB
    calls find those very jobs (field for field), none is left unused, and the
    bitstream is unchanged; SVTME_GLUE_PREFETCH=0 submits at the first SB call."""
    r = E.check(case, "ora", workdir)
    assert r["prefetched"] == r["pa_jobs"] + r["tf_jobs"] > 0 and r["prefetch_hits"] == r["prefetched"], r
    assert r["unused_jobs"] == 0 and r["fallback_sbs"] == 0
    r0 = E.check(case, "ora", workdir, env_extra={"SVTME_GLUE_PREFETCH": "0"})
    assert r0["prefetched"] == 0 and r0["pa_jobs"] == r["pa_jobs"] and r0["tf_jobs"] == r["tf_jobs"]


def _no_rtcd_registered(r):
    """Picture-job mode leaves every rtcd pointer to the encoder: the running
    encoder's pointers (the ten parity mode would replace, aom_dsp_rtcd.h:779,
    841-856, 863, 868) equal at exit what svt_aom_setup_rtcd_internal set before
    the first SB call (aom_dsp_rtcd.c:188, 501-528), and none is a HIP wrapper."""
    assert r["rtcd_checked"] == 10 and r["rtcd_changed"] == 0 and r["rtcd_hip"] == 0, r


@pytest.mark.skipif(not (E.available("ref") and E.available("ora")), reason="encoders built by oracle/encoder.mk")
def test_tf_jobs_and_redecimation_exercised(workdir):
    """At preset 8 temporal filtering runs: TF-ME jobs are served and the
    filtered pictures' pyramids are re-uploaded (svtme_picture_changed), at
    decimation time (eager uploads: every job finds its pictures resident)."""
    r = E.check("ra360_p12", "ora", workdir)
    assert r["tf_jobs"] > 0 and r["pa_jobs"] > 0 and r["invalidations"] > 0


@pytest.mark.skipif(not (E.available("ref") and E.available("ora")), reason="encoders built by oracle/encoder.mk")
@pytest.mark.parametrize("case", ["ra360_p12", "240p_p8_lowdelay"])
def test_job_time_uploads_only(case, workdir):
    """SVTME_GLUE_EAGER=0: no picture is uploaded at decimation time; every job
    uploads what it names on first use (the path eager uploads normally skip)."""
    r = E.check(case, "ora", workdir, {"SVTME_GLUE_EAGER": "0"})
    assert r["eager_uploads"] == 0 and r["uploads"] > 0 and r["fallback_sbs"] == 0
    assert r["verified_planes"] == 3 * r["uploads"]


@pytest.mark.gpu
@pytest.mark.skipif(not (E.available("ref") and E.available("gpu")), reason="encoders built by oracle/encoder.mk")
@pytest.mark.parametrize("case", GPU_CASES)
def test_bitstream_identical_gpu(case, workdir):
    r = E.check(case, "gpu", workdir)
    assert r["backend"] == 1 and r["sbs"] > 0 and r["fallback_sbs"] == 0
    _no_rtcd_registered(r)
    print(f"\n{case}: ref {r['ref_seconds']} s, GPU-ME encoder {r['glue_seconds']} s, {r['pa_jobs']} PA + "
          f"{r['tf_jobs']} TF jobs, {r['sbs']} SBs, served {r['served_sb_per_s'] / 1e6:.2f} M SB/s "
          f"(busy {r['busy_ms']} ms, mean job {r['job_latency_ms']} ms, up to {r['max_inflight']} in flight), "
          f"md5 {r['md5']}")
