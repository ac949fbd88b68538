"""svtme — Python host mirror of the MI355X open-loop motion-estimation stage.

ctypes bindings of include/svtme.h (libsvtme.so, the HIP product), plus the
same-ABI test checkers (oracle/liboracle.so, oracle/_ref/libsvtref.so) and the
synthetic generator (libsvtme_synth.so). The structures mirror the reference's
MeContext controls (Source/Lib/Codec/me_context.h:280-509) and ME results
(me_sb_results.h:28-52); names and meanings follow the reference.

Product entry points never fall back to a CPU path: if libsvtme.so is missing or
HIP fails, they raise.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)

PU_COUNT = 85
MAX_SAD_VALUE = 128 * 128 * 255
MAX_TICKETS = 64  # SVTME_MAX_TICKETS (include/svtme.h; tests/test_abi.py checks it)
PAD_FULL, PAD_QUARTER, PAD_SIXTEENTH = 72, 32, 16
SUB_SAD_SEARCH, FULL_SAD_SEARCH = 0, 1
ME_MCTF, ME_OPEN_LOOP = 1, 3  # EbMeType (me_context.h:44-51)
# kernel-path selection bits (include/svtme.h SVTME_PATH_*)
PATH_NO_FUSED_HME, PATH_NO_L1_FULL, PATH_NO_L0_FULL, PATH_NO_FP_WIDE, PATH_SPLIT_PASS = 1, 2, 4, 8, 16
# EbInputResolution (definitions.h:2079-2085)
RES_240P, RES_360P, RES_480P, RES_720P, RES_1080P, RES_4K, RES_8K = range(7)


# ----------------------------------------------------------------------------
# C structures (layout identical to include/svtme.h)
# ----------------------------------------------------------------------------
class Area(C.Structure):
    _fields_ = [("width", C.c_uint16), ("height", C.c_uint16)]


class AreaMinMax(C.Structure):
    _fields_ = [("sa_min", Area), ("sa_max", Area)]


class Controls(C.Structure):
    _fields_ = [
        ("hme_search_method", C.c_uint8),
        ("me_search_method", C.c_uint8),
        ("enable_hme_flag", C.c_uint8),
        ("enable_hme_level0_flag", C.c_uint8),
        ("enable_hme_level1_flag", C.c_uint8),
        ("enable_hme_level2_flag", C.c_uint8),
        ("num_hme_sa_w", C.c_uint8),
        ("num_hme_sa_h", C.c_uint8),
        ("hme_l0_sa", AreaMinMax),
        ("hme_l1_sa", Area),
        ("hme_l2_sa", Area),
        ("me_sa", AreaMinMax),
        ("enable_me_hme_ref_pruning", C.c_uint8),
        ("pad0", C.c_uint8),
        ("prune_ref_if_hme_sad_dev_bigger_than_th", C.c_uint16),
        ("prune_ref_if_me_sad_dev_bigger_than_th", C.c_uint16),
        ("zz_sad_pct", C.c_uint16),
        ("zz_sad_th", C.c_uint32),
        ("phme_sad_th", C.c_uint32),
        ("phme_sad_pct", C.c_uint16),
        ("enable_me_sr_adjustment", C.c_uint8),
        ("distance_based_hme_resizing", C.c_uint8),
        ("reduce_me_sr_based_on_mv_length_th", C.c_uint16),
        ("stationary_hme_sad_abs_th", C.c_uint16),
        ("stationary_me_sr_divisor", C.c_uint16),
        ("reduce_me_sr_based_on_hme_sad_abs_th", C.c_uint16),
        ("me_sr_divisor_for_low_hme_sad", C.c_uint16),
        ("mv_sa_adj_enabled", C.c_uint8),
        ("mv_sa_adj_nearest_ref_only", C.c_uint8),
        ("mv_sa_adj_mv_size_th", C.c_uint16),
        ("mv_sa_adj_sa_multiplier", C.c_uint16),
        ("me_8x8_var_enabled", C.c_uint8),
        ("pad1", C.c_uint8),
        ("me_sr_div4_th", C.c_uint32),
        ("me_sr_div2_th", C.c_uint32),
        ("me_sr_mult2_th", C.c_uint32),
        ("prehme_enable", C.c_uint8),
        ("prehme_skip_search_line", C.c_uint8),
        ("prehme_l1_early_exit", C.c_uint8),
        ("pad2", C.c_uint8),
        ("prehme_sa_cfg", AreaMinMax * 2),
        ("prune_me_candidates_th", C.c_int32),
        ("use_best_unipred_cand_only", C.c_uint8),
        ("reduce_hme_l0_sr_th_min", C.c_uint8),
        ("reduce_hme_l0_sr_th_max", C.c_uint8),
        ("pad3", C.c_uint8),
        ("me_early_exit_th", C.c_uint32),
        ("me_safe_limit_zz_th", C.c_uint32),
        ("prev_me_stage_based_exit_th", C.c_uint32),
    ]

    @staticmethod
    def from_dict(d: dict) -> "Controls":
        """Inverse of as_dict (golden fixtures store controls as dicts)."""
        c = Controls()
        for name, v in d.items():
            cur = getattr(c, name)
            if isinstance(cur, AreaMinMax):
                cur.sa_min.width, cur.sa_min.height = v[0]
                cur.sa_max.width, cur.sa_max.height = v[1]
            elif isinstance(cur, Area):
                cur.width, cur.height = v
            elif name == "prehme_sa_cfg":
                for a, vv in zip(cur, v):
                    a.sa_min.width, a.sa_min.height = vv[0]
                    a.sa_max.width, a.sa_max.height = vv[1]
            else:
                setattr(c, name, v)
        return c

    def as_dict(self):
        out = {}
        for name, _ in self._fields_:
            if name.startswith("pad"):
                continue
            v = getattr(self, name)
            if isinstance(v, AreaMinMax):
                v = ((v.sa_min.width, v.sa_min.height), (v.sa_max.width, v.sa_max.height))
            elif isinstance(v, Area):
                v = (v.width, v.height)
            elif name == "prehme_sa_cfg":
                v = tuple(((a.sa_min.width, a.sa_min.height), (a.sa_max.width, a.sa_max.height)) for a in v)
            out[name] = v
        return out


class Job(C.Structure):
    _fields_ = [
        ("picture_number", C.c_uint64),
        ("width", C.c_uint32),
        ("height", C.c_uint32),
        ("ref_picture_number", (C.c_uint64 * 4) * 2),
        ("num_lists", C.c_uint8),
        ("num_refs", C.c_uint8 * 2),
        ("temporal_layer_index", C.c_uint8),
        ("is_ref", C.c_uint8),
        ("hierarchical_levels", C.c_uint8),
        ("similar_brightness_refs", C.c_uint8),
        ("enable_me_8x8", C.c_uint8),
        ("enable_me_16x16", C.c_uint8),
        ("max_cand", C.c_uint8),
        ("max_refs", C.c_uint8),
        ("max_l0", C.c_uint8),
        ("only_l_bwd", C.c_uint8),
        ("input_resolution", C.c_uint8),
        ("gm_enabled", C.c_uint8),
        ("gm_use_distance_based_active_th", C.c_uint8),
        ("me_type", C.c_uint8),
        ("pad", C.c_uint8),
        ("tf_me_exit_th", C.c_uint16),
        ("sb_begin", C.c_uint32),
        ("sb_count", C.c_uint32),
        ("ctrl", Controls),
    ]


class Pyr(C.Structure):
    _fields_ = [("full", C.c_void_p), ("quarter", C.c_void_p), ("sixteenth", C.c_void_p)]


REF_RECORD_DTYPE = np.dtype(
    [
        ("best_sad", "<u4", (PU_COUNT,)),
        ("best_mv", "<u4", (PU_COUNT,)),
        ("hme_sad", "<u8"),
        ("hme_sc_x", "<i2"),
        ("hme_sc_y", "<i2"),
        ("zz_sad", "<u4"),
        ("searched", "u1"),
        ("do_ref", "u1"),
        ("tf_early_exit", "u1"),
        ("pad", "u1", (5,)),
    ]
)
assert REF_RECORD_DTYPE.itemsize == 704

SB_RESULT_DTYPE = np.dtype(
    [
        ("total_me_candidate_index", "u1", (PU_COUNT,)),
        ("pad0", "u1", (3,)),
        ("me_candidate_array", "u1", (PU_COUNT, 23)),
        ("pad1", "u1", (1,)),
        ("me_mv_array", "<u4", (PU_COUNT, 7)),
        ("me_distortion", "<u4", (PU_COUNT,)),
        ("me_8x8_cost_variance", "<u4"),
        ("rc_me_distortion", "<u4"),
        ("me_64x64_distortion", "<u4"),
        ("me_32x32_distortion", "<u4"),
        ("me_16x16_distortion", "<u4"),
        ("me_8x8_distortion", "<u4"),
        ("stationary_block_present", "u1"),
        ("rc_me_allow_gm", "u1"),
        ("pad2", "u1", (6,)),
    ]
)


class PackLayout(C.Structure):
    """svtme_pack_layout (include/svtme.h): the packed host output of a job."""
    _fields_ = [("n_pus", C.c_uint16), ("max_cand", C.c_uint8), ("max_refs", C.c_uint8),
                ("full_records", C.c_uint8), ("sb_results", C.c_uint8), ("pad", C.c_uint8 * 2)]


TAIL_BYTES = 24  # svtme_record_tail: the last 24 bytes of svtme_ref_record


def packed_sb_bytes(L: PackLayout, R: int) -> int:
    """svtme_packed_sb_bytes (include/svtme.h)."""
    b = R * (REF_RECORD_DTYPE.itemsize if L.full_records else TAIL_BYTES)
    if L.sb_results:
        b += 4 * (6 + PU_COUNT) + 4 * L.n_pus * L.max_refs + 4 + L.n_pus * (1 + L.max_cand)
    return (b + 15) & ~15


def pack_outputs(recs: np.ndarray, sbr, L: PackLayout) -> bytes:
    """The packed bytes of a job's outputs (records [n_sb][R], SB results [n_sb]),
    restated in numpy from the layout include/svtme.h documents."""
    n_sb, R = recs.shape
    stride = packed_sb_bytes(L, R)
    out = bytearray(n_sb * stride)
    raw = recs.tobytes()
    rs = REF_RECORD_DTYPE.itemsize
    for k in range(n_sb):
        o = k * stride
        for r in range(R):
            rec = raw[(k * R + r) * rs:(k * R + r + 1) * rs]
            part = rec if L.full_records else rec[rs - TAIL_BYTES:]
            out[o:o + len(part)] = part
            o += len(part)
        if L.sb_results:
            s = sbr[k]
            v = np.array([s["me_8x8_cost_variance"], s["rc_me_distortion"], s["me_64x64_distortion"],
                          s["me_32x32_distortion"], s["me_16x16_distortion"], s["me_8x8_distortion"]], "<u4")
            for part in (v.tobytes(), s["me_distortion"].astype("<u4").tobytes(),
                         np.ascontiguousarray(s["me_mv_array"][:L.n_pus, :L.max_refs]).astype("<u4").tobytes(),
                         bytes([int(s["stationary_block_present"]), int(s["rc_me_allow_gm"]), 0, 0]),
                         s["total_me_candidate_index"][:L.n_pus].tobytes(),
                         np.ascontiguousarray(s["me_candidate_array"][:L.n_pus, :L.max_cand]).tobytes()):
                out[o:o + len(part)] = part
                o += len(part)
    return bytes(out)


def sb_total(width: int, height: int) -> int:
    return ((width + 63) // 64) * ((height + 63) // 64)


def align8(v: int) -> int:
    return (v + 7) & ~7


def ref_slots(job: Job) -> int:
    return job.num_refs[0] + (job.num_refs[1] if job.num_lists == 2 else 0)


# ----------------------------------------------------------------------------
# Library loading
# ----------------------------------------------------------------------------
_LIBS: dict = {}


def _load(path: str, what: str):
    if path in _LIBS:
        return _LIBS[path]
    if not os.path.exists(path):
        raise RuntimeError(f"{what} not built: {path} is missing (run __graft_entry__.build())")
    lib = C.CDLL(path)
    _LIBS[path] = lib
    return lib


def _proto_common(lib, prefix):
    f = getattr(lib, prefix + "_me")
    f.argtypes = [C.POINTER(Job), C.POINTER(Pyr), C.POINTER(Pyr), C.c_void_p, C.c_void_p, C.c_int]
    f.restype = C.c_int32
    f = getattr(lib, prefix + "_build_pyramid")
    f.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(Pyr)]
    f.restype = None


def load_oracle():
    # SVTME_ORACLE_LIB: a sanitizer build of the same sources (scripts/sanitize_cpu.sh)
    lib = _load(os.environ.get("SVTME_ORACLE_LIB") or os.path.join(REPO_DIR, "oracle", "liboracle.so"), "CPU oracle")
    if not hasattr(lib, "_svtme_protos"):
        _proto_common(lib, "svtora")
        lib._svtme_protos = True
    return lib


def load_ref():
    lib = _load(os.path.join(REPO_DIR, "oracle", "_ref", "libsvtref.so"), "reference harness")
    if not hasattr(lib, "_svtme_protos"):
        _proto_common(lib, "svtref")
        lib.svtref_set_simd.argtypes = [C.c_int]
        lib.svtref_derive_controls.argtypes = [C.c_int] * 6 + [C.POINTER(Controls)]
        lib.svtref_derive_controls_tf.argtypes = [C.c_int] * 4 + [C.POINTER(Controls)]
        lib._svtme_protos = True
    return lib


def load_synth():
    lib = _load(os.environ.get("SVTME_SYNTH_LIB") or os.path.join(PKG_DIR, "libsvtme_synth.so"), "synthetic generator")
    if not hasattr(lib, "_svtme_protos"):
        lib.svtme_synth_texture_size.argtypes = [C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        lib.svtme_synth_texture.argtypes = [C.c_uint32, C.c_uint32, C.c_void_p]
        lib.svtme_synth_frame_from_texture.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p,
                                                       C.c_uint32]
        lib.svtme_synth_frame10_from_texture.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p,
                                                         C.c_uint32]
        lib.svtme_synth_frame_mixed_from_texture.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32,
                                                             C.c_void_p, C.c_uint32]
        lib._svtme_protos = True
    return lib


# ----------------------------------------------------------------------------
# Synthetic pictures
# ----------------------------------------------------------------------------
class Synth:
    """Deterministic pan of one texture; frame(t) returns an (h, w) uint8 array."""

    def __init__(self, width: int, height: int):
        self.w, self.h = width, height
        lib = load_synth()
        tw, th = C.c_uint32(), C.c_uint32()
        lib.svtme_synth_texture_size(width, height, C.byref(tw), C.byref(th))
        self.tex = np.empty((th.value, tw.value), np.uint8)
        lib.svtme_synth_texture(width, height, self.tex.ctypes.data)

    def frame(self, t: int) -> np.ndarray:
        out = np.empty((self.h, self.w), np.uint8)
        load_synth().svtme_synth_frame_from_texture(self.tex.ctypes.data, self.w, self.h, t, out.ctypes.data, self.w)
        return out

    def frame_mixed(self, t: int) -> np.ndarray:
        """Per-region motion (static .. beyond the search range) and noise regions."""
        out = np.empty((self.h, self.w), np.uint8)
        load_synth().svtme_synth_frame_mixed_from_texture(self.tex.ctypes.data, self.w, self.h, t, out.ctypes.data,
                                                          self.w)
        return out

    def frame10(self, t: int) -> np.ndarray:
        out = np.empty((self.h, self.w), np.uint16)
        load_synth().svtme_synth_frame10_from_texture(self.tex.ctypes.data, self.w, self.h, t, out.ctypes.data,
                                                      self.w)
        return out


def test_frames(kind: str, w: int, h: int, ts) -> dict:
    """Deterministic test content {t: luma plane} shared by the parity tests and
    the golden-fixture generator: a panning texture ("pan"; "vpan" / "hpan":
    fast vertical / horizontal motion), i.i.d. noise,
    flat, saturated (0/255) and moving stripes (exact ties everywhere)."""
    ts = list(ts)
    if kind == "pan":
        syn = Synth(w, h)
        return {t: syn.frame(t) for t in ts}
    if kind in ("vpan", "hpan"):  # 120 px per picture, vertical / horizontal (wraps around)
        base = Synth(w, h).frame(0)
        return {t: np.roll(base, 120 * t, axis=0 if kind == "vpan" else 1) for t in ts}
    rng = np.random.default_rng(1234)
    if kind == "noise":
        return {t: rng.integers(0, 256, (h, w), dtype=np.uint8) for t in ts}
    if kind == "flat":
        return {t: np.full((h, w), 128, np.uint8) for t in ts}
    if kind == "sat":
        return {t: (rng.integers(0, 2, (h, w)) * 255).astype(np.uint8) for t in ts}
    if kind == "stripes":
        base = ((np.arange(w)[None, :] // 4 + np.arange(h)[:, None] // 8) % 2 * 200).astype(np.uint8)
        return {t: np.roll(base, t, axis=1) for t in ts}
    raise ValueError(kind)


def case_job(ctrl: Controls, w: int, h: int, cur: int, l0, l1, tl: int, gm: bool = False, is_ref: bool = True,
             e8=None, sb_begin: int = 0, sb_count: int = 0, **kw) -> Job:
    """The job of one test case: references ordered as given, lists sized to them
    (kw: me_type / tf_me_exit_th for temporal-filtering jobs)."""
    res = input_resolution_of(w, h)
    return make_job(w, h, ctrl, cur, l0, l1, temporal_layer_index=tl, is_ref=is_ref,
                    enable_me_8x8=(res <= RES_720P) if e8 is None else e8,
                    ref_count_used=(max(len(l0), 1), len(l1)), gm_enabled=gm, sb_begin=sb_begin, sb_count=sb_count,
                    **kw)


def run_case_checker(kind: str, w: int, h: int, ctrl: Controls, cur: int, l0, l1, tl: int, checker: str = "oracle",
                     nthreads: int = 8, **kw):
    """One picture of test content through a CPU checker -> (records, sb_results)."""
    frames = test_frames(kind, w, h, sorted(set([cur] + list(l0) + list(l1))))
    pyr = {t: build_host_pyramid(f, checker) for t, f in frames.items()}
    refs = {}
    for i, t in enumerate(l0):
        refs[(0, i)] = pyr[t]
    for i, t in enumerate(l1):
        refs[(1, i)] = pyr[t]
    job = case_job(ctrl, w, h, cur, l0, l1, tl, **kw)
    return run_checker(job, pyr[cur], refs, checker, nthreads=nthreads)


# ----------------------------------------------------------------------------
# Host-side pyramids (for the CPU checkers)
# ----------------------------------------------------------------------------
@dataclass
class HostPyramid:
    width: int
    height: int
    full: np.ndarray
    quarter: np.ndarray
    sixteenth: np.ndarray
    pyr: Pyr = field(default=None)

    @staticmethod
    def alloc(width: int, height: int) -> "HostPyramid":
        W, H = align8(width), align8(height)
        full = np.zeros((H + 2 * PAD_FULL, W + 2 * PAD_FULL), np.uint8)
        quarter = np.zeros((H // 2 + 2 * PAD_QUARTER, W // 2 + 2 * PAD_QUARTER), np.uint8)
        six = np.zeros((H // 4 + 2 * PAD_SIXTEENTH, W // 4 + 2 * PAD_SIXTEENTH), np.uint8)
        p = HostPyramid(W, H, full, quarter, six)
        p.pyr = Pyr(full.ctypes.data, quarter.ctypes.data, six.ctypes.data)
        return p


def build_host_pyramid(y: np.ndarray, checker: str = "oracle") -> HostPyramid:
    y = np.ascontiguousarray(y)
    if y.dtype == np.uint16:  # 10-bit: search the MSB plane (enc_handle.c:4964-4972)
        y = (y >> 2).astype(np.uint8)
    h, w = y.shape
    p = HostPyramid.alloc(w, h)
    lib = load_oracle() if checker == "oracle" else load_ref()
    fn = lib.svtora_build_pyramid if checker == "oracle" else lib.svtref_build_pyramid
    fn(y.ctypes.data, w, w, h, C.byref(p.pyr))
    return p


def run_checker(job: Job, cur: HostPyramid, refs: dict, checker: str = "oracle", nthreads: int = 1,
                with_sb_results: bool = True):
    """refs: {(list, ref): HostPyramid}. Returns (ref_records[sb, R], sb_results[sb] or None)."""
    total = sb_total(job.width, job.height)
    count = job.sb_count if job.sb_count else total - job.sb_begin
    R = ref_slots(job)
    recs = np.zeros((count, R), REF_RECORD_DTYPE)
    sbr = np.zeros(count, SB_RESULT_DTYPE) if with_sb_results else None
    arr = (Pyr * 8)()
    for (l, r), p in refs.items():
        arr[l * 4 + r] = p.pyr
    if checker == "oracle":
        lib = load_oracle()
        st = lib.svtora_me(C.byref(job), C.byref(cur.pyr), arr, recs.ctypes.data,
                           sbr.ctypes.data if sbr is not None else None, nthreads)
    else:
        lib = load_ref()
        st = lib.svtref_me(C.byref(job), C.byref(cur.pyr), arr, recs.ctypes.data,
                           sbr.ctypes.data if sbr is not None else None, nthreads)
    if st != 0:
        raise RuntimeError(f"{checker} ME failed: status 0x{st & 0xffffffff:08x}")
    return recs, sbr


# ----------------------------------------------------------------------------
# Controls and jobs
# ----------------------------------------------------------------------------
def ref_derive_controls(enc_mode: int, qp: int, input_resolution: int, temporal_layer_index: int,
                        hierarchical_levels: int = 5, frame_rate_q16: int = 30 << 16) -> Controls:
    c = Controls()
    load_ref().svtref_derive_controls(enc_mode, qp, input_resolution, temporal_layer_index, hierarchical_levels,
                                      frame_rate_q16, C.byref(c))
    return c


def derive_controls(enc_mode: int, qp: int, input_resolution: int, temporal_layer_index: int,
                    hierarchical_levels: int = 5, frame_rate_q16: int = 30 << 16) -> Controls:
    """The product's restatement of svt_aom_sig_deriv_me (enc_mode_config.c:671-808)."""
    c = Controls()
    lib = load_product()
    lib.svtme_derive_controls(enc_mode, qp, input_resolution, temporal_layer_index, hierarchical_levels,
                              frame_rate_q16, C.byref(c))
    return c


def derive_controls_tf(hme_me_level: int, qp_opt: int, qp: int, input_resolution: int) -> Controls:
    """The product's restatement of the TF-ME controls (svt_aom_sig_deriv_me_tf,
    enc_mode_config.c:814-854) for a temporal-filtering (ME_MCTF) job."""
    c = Controls()
    load_product().svtme_derive_controls_tf(hme_me_level, qp_opt, qp, input_resolution, C.byref(c))
    return c


def ref_derive_controls_tf(hme_me_level: int, qp_opt: int, qp: int, input_resolution: int) -> Controls:
    c = Controls()
    load_ref().svtref_derive_controls_tf(hme_me_level, qp_opt, qp, input_resolution, C.byref(c))
    return c


def input_resolution_of(width: int, height: int) -> int:
    """svt_aom_derive_input_resolution (sequence_control_set.c:113-131) on the
    8-aligned luma size (resource_coordination_process.c:689)."""
    px = align8(width) * align8(height)
    for th, res in ((0x28500, RES_240P), (0x4CE00, RES_360P), (0xA1400, RES_480P), (0x16DA00, RES_720P),
                    (0x535200, RES_1080P), (0x140A000, RES_4K)):
        if px < th:
            return res
    return RES_8K


def max_allocated_me_refs(l0: int, l1: int):
    """pcs.c:91-96 svt_aom_get_max_allocated_me_refs -> (max_refs, max_cand)."""
    return l0 + l1, l0 + l1 + (l0 * l1) + (l0 - 1) + (1 if l1 == 3 else 0)


def make_job(width: int, height: int, ctrl: Controls, picture_number: int, refs_l0=(), refs_l1=(),
             temporal_layer_index: int = 1, is_ref: bool = True, hierarchical_levels: int = 5,
             enable_me_8x8: bool = False, input_resolution: int | None = None, ref_count_used=(2, 2),
             only_l_bwd: bool = True, gm_enabled: bool = False, sb_begin: int = 0, sb_count: int = 0,
             me_type: int = ME_OPEN_LOOP, tf_me_exit_th: int = 0) -> Job:
    j = Job()
    j.picture_number = picture_number
    j.width, j.height = align8(width), align8(height)
    for i, p in enumerate(refs_l0):
        j.ref_picture_number[0][i] = p
    for i, p in enumerate(refs_l1):
        j.ref_picture_number[1][i] = p
    j.num_lists = 2 if len(refs_l1) else 1
    j.num_refs[0] = len(refs_l0)
    j.num_refs[1] = len(refs_l1)
    j.temporal_layer_index = temporal_layer_index
    j.is_ref = 1 if is_ref else 0
    j.hierarchical_levels = hierarchical_levels
    j.similar_brightness_refs = 0
    j.enable_me_8x8 = 1 if enable_me_8x8 else 0
    j.enable_me_16x16 = 1
    mr, mc = max_allocated_me_refs(*ref_count_used)
    j.max_cand, j.max_refs, j.max_l0 = mc, mr, ref_count_used[0]
    j.only_l_bwd = 1 if only_l_bwd else 0
    j.input_resolution = input_resolution if input_resolution is not None else input_resolution_of(width, height)
    j.gm_enabled = 1 if gm_enabled else 0
    j.sb_begin, j.sb_count = sb_begin, sb_count
    j.me_type, j.tf_me_exit_th = me_type, tf_me_exit_th
    j.ctrl = ctrl
    return j


# ----------------------------------------------------------------------------
# Product library (HIP): loaded lazily; raises if absent
# ----------------------------------------------------------------------------
def product_lib_path() -> str:
    # SVTME_LIB: a diagnostic build of the same sources (e.g. scripts/hme_stamps.py)
    return os.environ.get("SVTME_LIB") or os.path.join(PKG_DIR, "libsvtme.so")


def load_product():
    return _job_api_protos(_load(product_lib_path(), "HIP product library libsvtme.so"))


def load_oracle_job():
    """oracle/liboraclejob.so: the job API over the CPU oracle (test infrastructure,
    the encoder tests' backend); the entry points it implements get prototypes."""
    return _job_api_protos(_load(os.path.join(REPO_DIR, "oracle", "liboraclejob.so"), "oracle job API"))


def _proto(lib, name, attr, val):
    if hasattr(lib, name):  # (the oracle job API implements a subset)
        setattr(getattr(lib, name), attr, val)


def _job_api_protos(lib):
    if not hasattr(lib, "_svtme_protos"):
        vp = C.c_void_p
        _proto(lib, "svtme_ctx_create", "argtypes", [C.c_int, C.POINTER(vp)])
        _proto(lib, "svtme_ctx_create", "restype", C.c_int32)
        _proto(lib, "svtme_ctx_destroy", "argtypes", [vp])
        _proto(lib, "svtme_ctx_destroy", "restype", None)
        _proto(lib, "svtme_picture_upload", "argtypes", [vp, C.c_uint64, vp, C.c_uint32, C.c_uint32, C.c_uint32])
        _proto(lib, "svtme_picture_upload", "restype", C.c_int32)
        _proto(lib, "svtme_picture_upload_10bit", "argtypes", [vp, C.c_uint64, vp, C.c_uint32, C.c_uint32, C.c_uint32])
        _proto(lib, "svtme_picture_upload_10bit", "restype", C.c_int32)
        _proto(lib, "svtme_picture_upload_async", "argtypes", [vp, C.c_uint64, vp, C.c_uint32, C.c_uint32, C.c_uint32])
        _proto(lib, "svtme_picture_upload_async", "restype", C.c_int32)
        _proto(lib, "svtme_picture_upload_copy_async", "argtypes", [vp, C.c_uint64, vp, C.c_uint32, C.c_uint32,
                                                                    C.c_uint32])
        _proto(lib, "svtme_picture_upload_copy_async", "restype", C.c_int32)
        _proto(lib, "svtme_reserve_pictures", "argtypes", [vp, C.c_uint32, C.c_uint32, C.c_uint32])
        _proto(lib, "svtme_reserve_pictures", "restype", C.c_int32)
        _proto(lib, "svtme_picture_upload_device", "argtypes", [vp, C.c_uint64, vp, C.c_uint32, C.c_uint32, C.c_uint32])
        _proto(lib, "svtme_picture_upload_device", "restype", C.c_int32)
        _proto(lib, "svtme_picture_upload_device_async", "argtypes", [vp, C.c_uint64, vp, C.c_uint32, C.c_uint32,
                                                                      C.c_uint32])
        _proto(lib, "svtme_picture_upload_device_async", "restype", C.c_int32)
        _proto(lib, "svtme_upload_stream", "argtypes", [vp])
        _proto(lib, "svtme_upload_stream", "restype", vp)
        _proto(lib, "svtme_picture_invalidate", "argtypes", [vp, C.c_uint64, vp, C.c_uint32, C.c_uint32, C.c_uint32])
        _proto(lib, "svtme_picture_invalidate", "restype", C.c_int32)
        _proto(lib, "svtme_picture_release", "argtypes", [vp, C.c_uint64])
        _proto(lib, "svtme_picture_release", "restype", C.c_int32)
        _proto(lib, "svtme_picture_download", "argtypes", [vp, C.c_uint64, C.c_int, vp, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)])
        _proto(lib, "svtme_picture_download", "restype", C.c_int32)
        _proto(lib, "svtme_submit_picture", "argtypes", [vp, C.POINTER(Job), vp, vp])
        _proto(lib, "svtme_submit_picture", "restype", C.c_int32)
        _proto(lib, "svtme_submit_picture_async", "argtypes", [vp, C.POINTER(Job)])
        _proto(lib, "svtme_submit_picture_async", "restype", C.c_int32)
        _proto(lib, "svtme_sync", "argtypes", [vp])
        _proto(lib, "svtme_sync", "restype", C.c_int32)
        _proto(lib, "svtme_fetch", "argtypes", [vp, vp, vp])
        _proto(lib, "svtme_fetch", "restype", C.c_int32)
        _proto(lib, "svtme_submit_picture_device", "argtypes", [vp, C.POINTER(Job), vp, vp])
        _proto(lib, "svtme_submit_picture_device", "restype", C.c_int32)
        _proto(lib, "svtme_submit_picture_packed_async", "argtypes", [vp, C.c_uint32, C.POINTER(Job), C.POINTER(PackLayout), vp, C.POINTER(C.c_uint64)])
        _proto(lib, "svtme_submit_picture_packed_async", "restype", C.c_int32)
        _proto(lib, "svtme_ticket_wait", "argtypes", [vp, C.c_uint64])
        _proto(lib, "svtme_ticket_wait", "restype", C.c_int32)
        _proto(lib, "svtme_host_alloc", "argtypes", [C.c_uint64])
        _proto(lib, "svtme_host_alloc", "restype", vp)
        _proto(lib, "svtme_host_free", "argtypes", [vp])
        _proto(lib, "svtme_host_free", "restype", None)
        _proto(lib, "svtme_reserve", "argtypes", [vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32])
        _proto(lib, "svtme_reserve", "restype", C.c_int32)
        _proto(lib, "svtme_set_paths", "argtypes", [vp, C.c_uint32])
        _proto(lib, "svtme_set_paths", "restype", C.c_int32)
        _proto(lib, "svtme_set_timing", "argtypes", [vp, C.c_int])
        _proto(lib, "svtme_set_timing", "restype", C.c_int32)
        _proto(lib, "svtme_timing_read", "argtypes", [vp, C.POINTER(C.c_float)])
        _proto(lib, "svtme_timing_read", "restype", C.c_uint32)
        _proto(lib, "svtme_submit_batch_device", "argtypes", [vp, C.POINTER(Job), C.c_uint32, C.POINTER(vp), C.POINTER(vp)])
        _proto(lib, "svtme_submit_batch_device", "restype", C.c_int32)
        _proto(lib, "svtme_submit_batch_device_lane", "argtypes", [vp, C.c_uint32, C.POINTER(Job), C.c_uint32, C.POINTER(vp), C.POINTER(vp)])
        _proto(lib, "svtme_submit_batch_device_lane", "restype", C.c_int32)
        _proto(lib, "svtme_lane_stream", "argtypes", [vp, C.c_uint32])
        _proto(lib, "svtme_lane_stream", "restype", vp)
        _proto(lib, "svtme_device_records", "argtypes", [vp, C.POINTER(C.c_uint64)])
        _proto(lib, "svtme_device_records", "restype", vp)
        _proto(lib, "svtme_stream", "argtypes", [vp])
        _proto(lib, "svtme_stream", "restype", vp)
        _proto(lib, "svtme_rtcd_failed", "argtypes", [])
        _proto(lib, "svtme_rtcd_failed", "restype", C.c_int)
        _proto(lib, "svtme_last_error", "argtypes", [])
        _proto(lib, "svtme_last_error", "restype", C.c_char_p)
        _proto(lib, "svtme_derive_controls", "argtypes", [C.c_int] * 6 + [C.POINTER(Controls)])
        _proto(lib, "svtme_derive_controls", "restype", None)
        _proto(lib, "svtme_derive_controls_tf", "argtypes", [C.c_int] * 4 + [C.POINTER(Controls)])
        _proto(lib, "svtme_derive_controls_tf", "restype", None)
        _proto(lib, "svtme_sb_total", "argtypes", [C.c_uint32, C.c_uint32])
        _proto(lib, "svtme_sb_total", "restype", C.c_uint32)
        lib._svtme_protos = True
    return lib


class GpuME:
    """The picture-level job API on one HIP device (no CPU fallback)."""

    def __init__(self, device: int = 0, lib=None):
        self.lib = lib or load_product()
        self.ctx = C.c_void_p()
        self._check(self.lib.svtme_ctx_create(device, C.byref(self.ctx)), "svtme_ctx_create")

    def _check(self, st, what):
        if st != 0:
            msg = self.lib.svtme_last_error().decode(errors="replace")
            raise RuntimeError(f"{what} failed: status 0x{st & 0xffffffff:08x}: {msg}")

    def close(self):
        if self.ctx:
            self.lib.svtme_ctx_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload(self, picture_number: int, y: np.ndarray):
        y = np.ascontiguousarray(y)
        h, w = y.shape
        if y.dtype == np.uint16:
            self._check(self.lib.svtme_picture_upload_10bit(self.ctx, picture_number, y.ctypes.data, w, w, h),
                        "svtme_picture_upload_10bit")
        else:
            self._check(self.lib.svtme_picture_upload(self.ctx, picture_number, y.ctypes.data, w, w, h),
                        "svtme_picture_upload")

    def upload_async(self, picture_number: int, y, w: int = 0, h: int = 0, stride: int = 0):
        """Asynchronous 8-bit upload (svtme_picture_upload_async): `y` is a uint8
        array or a host pointer (then w, h, stride); keep it alive until sync."""
        if isinstance(y, np.ndarray):
            h, w = y.shape
            stride, ptr = w, y.ctypes.data
        else:
            ptr = y
        self._check(self.lib.svtme_picture_upload_async(self.ctx, picture_number, ptr, stride or w, w, h),
                    "svtme_picture_upload_async")

    def upload_copy_async(self, picture_number: int, y, w: int = 0, h: int = 0, stride: int = 0):
        """svtme_picture_upload_copy_async: the rows are copied into the library's
        page-locked staging ring before the call returns; `y` may change after it."""
        if isinstance(y, np.ndarray):
            h, w = y.shape
            stride, ptr = w, y.ctypes.data
        else:
            ptr = y
        self._check(self.lib.svtme_picture_upload_copy_async(self.ctx, picture_number, ptr, stride or w, w, h),
                    "svtme_picture_upload_copy_async")

    def reserve_pictures(self, width: int, height: int, count: int):
        """svtme_reserve_pictures: `count` idle picture buffers of that size in the pool."""
        self._check(self.lib.svtme_reserve_pictures(self.ctx, width, height, count), "svtme_reserve_pictures")

    def upload_device(self, picture_number: int, dev_ptr: int, stride: int, w: int, h: int):
        self._check(self.lib.svtme_picture_upload_device(self.ctx, picture_number, dev_ptr, stride, w, h),
                    "svtme_picture_upload_device")

    def upload_device_async(self, picture_number: int, dev_ptr: int, stride: int, w: int, h: int):
        """svtme_picture_upload_device_async: the pyramid built on the upload stream."""
        self._check(self.lib.svtme_picture_upload_device_async(self.ctx, picture_number, dev_ptr, stride, w, h),
                    "svtme_picture_upload_device_async")

    def upload_stream(self) -> int:
        return self.lib.svtme_upload_stream(self.ctx) or 0

    def invalidate(self, picture_number: int, y: np.ndarray):
        """The resident picture's planes were replaced (TF re-decimation): rebuild."""
        y = np.ascontiguousarray(y)
        h, w = y.shape
        self._check(self.lib.svtme_picture_invalidate(self.ctx, picture_number, y.ctypes.data, w, w, h),
                    "svtme_picture_invalidate")

    def release(self, picture_number: int):
        self._check(self.lib.svtme_picture_release(self.ctx, picture_number), "svtme_picture_release")

    def download(self, picture_number: int, level: int) -> np.ndarray:
        stride, w, h, pad = C.c_uint32(), C.c_uint32(), C.c_uint32(), C.c_uint32()
        self._check(self.lib.svtme_picture_download(self.ctx, picture_number, level, None, C.byref(stride),
                                                    C.byref(w), C.byref(h), C.byref(pad)), "svtme_picture_download")
        out = np.empty((h.value + 2 * pad.value, stride.value), np.uint8)
        self._check(self.lib.svtme_picture_download(self.ctx, picture_number, level, out.ctypes.data,
                                                    C.byref(stride), C.byref(w), C.byref(h), C.byref(pad)),
                    "svtme_picture_download")
        return out

    def submit(self, job: Job, with_sb_results: bool = True):
        total = sb_total(job.width, job.height)
        count = job.sb_count if job.sb_count else total - job.sb_begin
        recs = np.zeros((count, ref_slots(job)), REF_RECORD_DTYPE)
        sbr = np.zeros(count, SB_RESULT_DTYPE) if with_sb_results else None
        self._check(self.lib.svtme_submit_picture(self.ctx, C.byref(job), recs.ctypes.data,
                                                  sbr.ctypes.data if sbr is not None else None),
                    "svtme_submit_picture")
        return recs, sbr

    def submit_async(self, job: Job):
        self._check(self.lib.svtme_submit_picture_async(self.ctx, C.byref(job)), "svtme_submit_picture_async")

    def submit_device(self, job: Job, d_records: int, d_sb: int | None = None):
        self._check(self.lib.svtme_submit_picture_device(self.ctx, C.byref(job), d_records, d_sb),
                    "svtme_submit_picture_device")

    def submit_packed(self, job: Job, layout: PackLayout, lane: int = 0, wait: bool = True):
        """svtme_submit_picture_packed_async into a page-locked buffer (svtme_host_alloc);
        returns (ticket, pointer, bytes), or the packed bytes when `wait`."""
        total = sb_total(job.width, job.height)
        count = job.sb_count if job.sb_count else total - job.sb_begin
        nbytes = count * packed_sb_bytes(layout, ref_slots(job))
        ptr = self.lib.svtme_host_alloc(nbytes)
        if not ptr:
            raise RuntimeError("svtme_host_alloc failed")
        t = C.c_uint64()
        st = self.lib.svtme_submit_picture_packed_async(self.ctx, lane, C.byref(job), C.byref(layout), ptr,
                                                        C.byref(t))
        if st != 0:
            self.lib.svtme_host_free(ptr)
            self._check(st, "svtme_submit_picture_packed_async")
        if not wait:
            return t.value, ptr, nbytes
        return self.wait_packed(t.value, ptr, nbytes)

    def wait_packed(self, ticket: int, ptr: int, nbytes: int) -> bytes:
        try:
            self._check(self.lib.svtme_ticket_wait(self.ctx, ticket), "svtme_ticket_wait")
            return C.string_at(ptr, nbytes)
        finally:
            self.lib.svtme_host_free(ptr)

    def reserve(self, width: int, height: int, max_refs: int = 8, tickets: int = 4):
        """svtme_reserve: size the lanes' scratch and the first `tickets` packed-job
        buffers for jobs up to width x height with max_refs reference slots."""
        self._check(self.lib.svtme_reserve(self.ctx, width, height, max_refs, tickets), "svtme_reserve")

    def set_paths(self, paths: int):
        """Kernel-path selection (SVTME_PATH_* bits; 0 = every specialised kernel)."""
        self._check(self.lib.svtme_set_paths(self.ctx, paths), "svtme_set_paths")

    def set_timing(self, enable: bool = True):
        self._check(self.lib.svtme_set_timing(self.ctx, 1 if enable else 0), "svtme_set_timing")

    def timing_read(self):
        """(submissions averaged, [ms of k_stage_a, k_stage_d, k_stage_b, k_stage_c1|c, k_stage_e])
        over the launches recorded since timing was enabled or last read."""
        ms = (C.c_float * 5)()
        n = self.lib.svtme_timing_read(self.ctx, ms)
        return int(n), [float(v) for v in ms]

    def submit_batch_device(self, jobs, d_records, d_sb=None, lane=None):
        """One launch per stage over several jobs (device outputs, asynchronous);
        lane: svtme_submit_batch_device_lane (None: the context stream, lane 0)."""
        n = len(jobs)
        arr = (Job * n)(*jobs)
        recs = (C.c_void_p * n)(*d_records)
        sbs = (C.c_void_p * n)(*d_sb) if d_sb is not None else None
        if lane is None:
            self._check(self.lib.svtme_submit_batch_device(self.ctx, arr, n, recs, sbs), "svtme_submit_batch_device")
        else:
            self._check(self.lib.svtme_submit_batch_device_lane(self.ctx, lane, arr, n, recs, sbs),
                        "svtme_submit_batch_device_lane")

    def lane_stream(self, lane: int) -> int:
        return self.lib.svtme_lane_stream(self.ctx, lane) or 0

    def submit_batch(self, jobs, with_sb_results: bool = True):
        """Batch submission with host outputs (tests): device buffers via torch."""
        import torch

        outs, d_recs, d_sb = [], [], []
        for job in jobs:
            total = sb_total(job.width, job.height)
            count = job.sb_count if job.sb_count else total - job.sb_begin
            r = torch.empty(count * ref_slots(job) * REF_RECORD_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
            sb = torch.empty(count * SB_RESULT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
            outs.append((r, sb, count, ref_slots(job)))
            d_recs.append(r.data_ptr())
            d_sb.append(sb.data_ptr())
        self.submit_batch_device(jobs, d_recs, d_sb if with_sb_results else None)
        self.sync()
        res = []
        for r, sb, count, R in outs:
            recs = np.frombuffer(r.cpu().numpy().tobytes(), REF_RECORD_DTYPE).reshape(count, R)
            sbr = np.frombuffer(sb.cpu().numpy().tobytes(), SB_RESULT_DTYPE).reshape(count) if with_sb_results else None
            res.append((recs, sbr))
        return res

    def sync(self):
        self._check(self.lib.svtme_sync(self.ctx), "svtme_sync")

    def fetch(self, job: Job, with_sb_results: bool = True):
        total = sb_total(job.width, job.height)
        count = job.sb_count if job.sb_count else total - job.sb_begin
        recs = np.zeros((count, ref_slots(job)), REF_RECORD_DTYPE)
        sbr = np.zeros(count, SB_RESULT_DTYPE) if with_sb_results else None
        self._check(self.lib.svtme_fetch(self.ctx, recs.ctypes.data, sbr.ctypes.data if sbr is not None else None),
                    "svtme_fetch")
        return recs, sbr

    def device_records(self):
        n = C.c_uint64()
        p = self.lib.svtme_device_records(self.ctx, C.byref(n))
        return p, n.value

    def stream(self) -> int:
        return self.lib.svtme_stream(self.ctx) or 0


# ----------------------------------------------------------------------------
# Record comparison
# ----------------------------------------------------------------------------
def compare_records(a: np.ndarray, b: np.ndarray, sa=None, sb=None) -> list:
    """Bit-exact comparison on the fields the reference defines; returns a list
    of human-readable mismatch descriptions (empty = identical)."""
    errs = []
    for f in ("searched", "do_ref", "tf_early_exit", "hme_sad", "hme_sc_x", "hme_sc_y", "zz_sad", "best_mv"):
        if not np.array_equal(a[f], b[f]):
            idx = np.argwhere(a[f] != b[f])[0]
            errs.append(f"{f} differs at {tuple(idx)}: {a[f][tuple(idx)]} vs {b[f][tuple(idx)]}")
    m = a["searched"].astype(bool)
    if not np.array_equal(a["best_sad"][m], b["best_sad"][m]):
        errs.append("best_sad differs on searched refs")
    if sa is not None and sb is not None:
        for f in SB_RESULT_DTYPE.names:
            if f.startswith("pad"):
                continue
            if not np.array_equal(sa[f], sb[f]):
                idx = np.argwhere(sa[f] != sb[f])[0]
                errs.append(f"sb.{f} differs at {tuple(idx)}")
    return errs


def records_checksum(recs: np.ndarray, sbr=None) -> str:
    import hashlib

    h = hashlib.sha256()
    r = recs.copy()
    r["best_sad"][~r["searched"].astype(bool)] = 0xFFFFFFFF
    r["pad"] = 0
    h.update(r.tobytes())
    if sbr is not None:
        s = sbr.copy()
        for f in ("pad0", "pad1", "pad2"):
            s[f] = 0
        h.update(s.tobytes())
    return h.hexdigest()
