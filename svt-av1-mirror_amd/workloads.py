"""The BASELINE.json configurations as picture jobs.

One definition shared by bench.py, the full-size parity tests and the golden
fixture generator (tests/golden/make_golden.py), so the benched workload is
exactly the one whose records are pinned against the reference.

  1080p_sa64  configs[1]: 1920x1080 p8, 1 ref, ME area override 64x64
  4k_p8       configs[2]: 3840x2160 p8, 4 refs (L0 d=1,2; L1 d=1,2) -- the headline
  4k10_p6     configs[3]: 3840x2160 10-bit p6 (MSB plane), refs as the encoder (1+1)
  8k_p8       configs[4]: 7680x4320 p8, 4 refs (sharded over GPUs in bench --mode band)
  4k_p8_mixed configs[2] on mixed-motion content (per-region motion and noise)
  4k_tf_p8    the temporal-filtering ME (ME_MCTF) of configs[2]'s encode (TF level 2 controls)
  ra360_p12   configs[0]: 640x360 p12, 30 pictures random access (ra_sequence)

Inputs are the integer PCG32 panning texture of SURVEY.md 8(d): current picture
t=8, references 7, 6 (list 0) and 9, 10 (list 1).
"""
from __future__ import annotations

import svtme as S

WORKLOADS = {
    "4k_p8": dict(w=3840, h=2160, mode=8, tl=1, l0=(7, 6), l1=(9, 10), windows="p8", ten_bit=False,
                  desc="3840x2160 8-bit preset 8, 4 refs (L0 d=1,2; L1 d=1,2), open-loop ME"),
    "1080p_sa64": dict(w=1920, h=1080, mode=8, tl=1, l0=(7,), l1=(), windows="p8_sa64", ten_bit=False, sa64=True,
                       desc="1920x1080 8-bit preset 8, 1 ref (L0 d=1), ME area override 64x64 "
                            "(8x8-variance resize and sr-adjust off: 4096 positions/SB), open-loop ME"),
    "4k10_p6": dict(w=3840, h=2160, mode=6, tl=1, l0=(7,), l1=(9,), windows="p6", ten_bit=True,
                    desc="3840x2160 10-bit preset 6 (8-bit MSB search), 2 refs, open-loop ME"),
    "8k_p8": dict(w=7680, h=4320, mode=8, tl=1, l0=(7, 6), l1=(9, 10), windows="p8", ten_bit=False,
                  desc="7680x4320 8-bit preset 8, 4 refs, open-loop ME"),
    # configs[2] on content whose motion varies across the picture (static regions take the zz early
    # exits, fast / out-of-range / noise regions the pruning and the worst-case windows)
    "4k_p8_mixed": dict(w=3840, h=2160, mode=8, tl=1, l0=(7, 6), l1=(9, 10), windows="p8", ten_bit=False,
                        content="mixed",
                        desc="3840x2160 8-bit preset 8, 4 refs (L0 d=1,2; L1 d=1,2), open-loop ME, mixed-motion "
                             "content (256x256 regions: static / slow / pan / fast / beyond range / noise)"),
    # temporal-filtering ME of configs[2]'s encode: the M8 tf_level 8 parameters (enc_handle.c:3125-3150:
    # hme_me_level 2 -> FULL-SAD HME L0 + L1, 8x8 full-pel, qp_opt; me_exit_th 16 x 16), central picture 8
    # against its nearest past picture (temporal_filtering.c:3127-3174)
    "4k_tf_p8": dict(w=3840, h=2160, tf=dict(level=2, qp_opt=1, qp=35, exit_th=16 * 16), tl=1, l0=(7,), l1=(),
                     windows="tf2", ten_bit=False,
                     desc="3840x2160 8-bit TF-ME (ME_MCTF) of preset 8 (hme_me_level 2: full-SAD HME, 8x8 "
                          "full-pel), central picture vs its nearest past picture"),
}
# the bench accepted "1080p_p8" in round 1
WORKLOADS["1080p_p8"] = WORKLOADS["1080p_sa64"]

# algorithmic bytes per SB = src 2688 + R x (nominal ref windows + 680 B out)
WINDOW_BYTES = {"p8": 16798, "p6": 38121, "p8_sa64": 28241,
                # TF level 2 (full rows): HME-L0 4 quadrants at 1/16 (48 x 32), HME-L1 4 x (16 + 32)^2 at 1/4,
                # full-pel (8 + 64)^2
                "tf2": 48 * 32 + 4 * 48 * 48 + 72 * 72}
# source bytes per SB the searches read (sub-sampled rows: 64x32 + 32x16 + 16x8; full rows for tf2)
SRC_BYTES = {"tf2": 64 * 64 + 32 * 32 + 16 * 16}
# absdiff operations per SB and reference (secondary, VALU-SAD roof)
ABSDIFF_PER_SB_REF = {"p8": 196608, "p6": 845824, "p8_sa64": 8536064,
                      # zz 64x32 + L0 4 x (16 x 8) x 16^2 + L1 4 x 16^2 x 32^2 + full-pel 64 x 64^2
                      "tf2": 2048 + 512 * 256 + 1024 * 1024 + 64 * 4096}
# of which the full-pel search: positions x 64x32 sub-sampled pixels (the 64x64 override: 4096 x 2048)
FULLPEL_ABSDIFF_PER_SB_REF = {"p8_sa64": 4096 * 2048}


def bytes_per_sb(windows: str, refs: int) -> int:
    return SRC_BYTES.get(windows, 2688) + refs * (WINDOW_BYTES[windows] + 680)


def workload_frame(name: str, syn: "S.Synth", t: int):
    """Picture t of the workload's content (uint16 plane for 10-bit)."""
    wl = WORKLOADS[name]
    if wl.get("content") == "mixed":
        return syn.frame_mixed(t)
    return syn.frame10(t) if wl["ten_bit"] else syn.frame(t)


def workload_frames(name: str) -> dict:
    """{t: luma plane} of the workload (uint16 planes for 10-bit)."""
    wl = WORKLOADS[name]
    syn = S.Synth(wl["w"], wl["h"])
    ts = sorted(set((8,) + tuple(wl["l0"]) + tuple(wl["l1"])))
    return {t: workload_frame(name, syn, t) for t in ts}


def workload_controls(name: str) -> S.Controls:
    wl = WORKLOADS[name]
    if wl.get("tf"):  # svt_aom_sig_deriv_me_tf + set_hme_search_params_mctf
        tf = wl["tf"]
        return S.derive_controls_tf(tf["level"], tf["qp_opt"], tf["qp"], S.input_resolution_of(wl["w"], wl["h"]))
    ctrl = S.derive_controls(wl["mode"], 35, S.input_resolution_of(wl["w"], wl["h"]), wl["tl"])
    if wl.get("sa64"):  # fixed 64x64 full-pel area
        ctrl.me_sa.sa_min.width = ctrl.me_sa.sa_min.height = 64
        ctrl.me_sa.sa_max.width = ctrl.me_sa.sa_max.height = 64
        ctrl.me_8x8_var_enabled = 0
        ctrl.enable_me_sr_adjustment = 0
    return ctrl


def workload_job(name: str, base: int = 0, sb_begin: int = 0, sb_count: int = 0) -> S.Job:
    """The picture job; picture numbers are base + t (t = 8 current, refs as listed)."""
    wl = WORKLOADS[name]
    res = S.input_resolution_of(wl["w"], wl["h"])
    tf = wl.get("tf")
    kw = dict(me_type=S.ME_MCTF, tf_me_exit_th=tf["exit_th"]) if tf else {}
    return S.make_job(wl["w"], wl["h"], workload_controls(name), base + 8, [base + t for t in wl["l0"]],
                      [base + t for t in wl["l1"]], temporal_layer_index=wl["tl"],
                      enable_me_8x8=(res <= S.RES_720P), ref_count_used=(3, 2), sb_begin=sb_begin,
                      sb_count=sb_count, **kw)


# ----------------------------------------------------------------------------
# configs[0]: 640x360 preset 12, 30 pictures, random access
# ----------------------------------------------------------------------------
# Temporal layer of each display position 1..16 of a five-level mini-GOP
# (five_level_hierarchical_pred_struct, pred_structure.c:218-282: GOP index i
# is display position i of the mini-GOP, index 0 being its base picture).
_FIVE_LEVEL_TL = {16: 0, 8: 1, 4: 2, 12: 2}
for _p in (2, 6, 10, 14):
    _FIVE_LEVEL_TL[_p] = 3
for _p in range(1, 16, 2):
    _FIVE_LEVEL_TL[_p] = 4


def ra_sequence(n: int = 30, mini_gop: int = 16, max_refs: int = 2):
    """[(picture, temporal_layer, l0 refs, l1 refs)] for pictures 1..n-1 of a
    random-access sequence (picture 0 is the key frame: no ME). References are
    the nearest already-coded pictures of a lower temporal layer: backward ones
    in list 0 and forward ones in list 1 (up to max_refs each), the base layer
    referencing previous base pictures only. This is the dependency shape of
    the hierarchical structure, not a restatement of the reference's RPS
    derivation: the ME parity it checks does not depend on which pictures are
    referenced."""
    seq = []
    last = n - 1
    for t in range(1, n):
        gop0 = ((t - 1) // mini_gop) * mini_gop
        pos = t - gop0
        tl = _FIVE_LEVEL_TL[pos]
        if t == last and tl != 0:
            tl = 0  # the last picture anchors the truncated final mini-GOP
        end = min(gop0 + mini_gop, last)  # forward references stay inside the mini-GOP
        if tl == 0:
            l0 = sorted([u for u in range(t) if _tl_of(u, n, mini_gop) == 0], reverse=True)[:max_refs]
            l1 = []
        else:
            lower = [u for u in range(0, end + 1) if u != t and _tl_of(u, n, mini_gop) < tl]
            l0 = sorted([u for u in lower if u < t], reverse=True)[:max_refs]
            l1 = sorted([u for u in lower if u > t])[:max_refs]
        seq.append((t, tl, tuple(l0), tuple(l1)))
    return seq


def _tl_of(u: int, n: int, mini_gop: int) -> int:
    if u == 0:
        return 0
    if u == n - 1:
        return 0
    return _FIVE_LEVEL_TL[u - ((u - 1) // mini_gop) * mini_gop]
