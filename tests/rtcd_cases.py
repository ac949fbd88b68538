"""Per-kernel rtcd cases (shared by the golden generator, the CPU oracle tests
and the GPU `*_hip` tests).

Each case is a deterministic function of its seed; `run(backend, case)` calls
one kernel with the reference signature through ctypes and returns its outputs
as numpy arrays. Backends are named by symbol prefix:

* "svt_"     + "_hip" suffix: the product (libsvtme.so, GPU);
* "svtora_"  : the CPU restatement (oracle/liboracle.so);
* "svtref_"  : the reference's own kernels compiled from source (oracle/_ref).

Shapes mirror the reference's SadTest coverage (test/SadTest.cc):
* unaligned pointers and odd strides (127);
* block widths 1..128;
* search areas up to 640 x 400;
* flat and saturated content (ties, extreme SADs).
"""
import ctypes as C

import numpy as np

U8P = C.POINTER(C.c_uint8)
U16P = C.POINTER(C.c_uint16)
U32P = C.POINTER(C.c_uint32)


def _u8(a):
    return a.ctypes.data_as(U8P)


def _u32(a):
    return a.ctypes.data_as(U32P)


def _content(rng, n, kind, hi=256, dtype=np.uint8):
    if kind == "flat":
        return np.full(n, hi // 2, dtype)
    if kind == "sat":
        return (rng.integers(0, 2, n) * (hi - 1)).astype(dtype)
    return rng.integers(0, hi, n, dtype=np.int64).astype(dtype)


# ----------------------------------------------------------------------------
# case lists
# ----------------------------------------------------------------------------
SAD_LOOP = [
    # (bw, bh, sa_w, sa_h, skip, sub, src_stride, ref_raw, ref_off, kind)
    (16, 8, 8, 100, 1, True, 32, 128, 3, "rand"),      # pre-HME v (1/16, sub, line skip)
    (16, 8, 32, 7, 1, True, 32, 130, 1, "rand"),       # pre-HME h
    (16, 8, 16, 4, 0, True, 32, 160, 2, "rand"),       # HME L0 quadrant
    (32, 16, 8, 3, 0, True, 64, 288, 1, "rand"),       # HME L1
    (64, 32, 8, 3, 0, True, 128, 512, 0, "rand"),      # HME L2
    (16, 16, 17, 9, 1, False, 127, 127, 5, "rand"),    # odd strides, full rows, skip
    (12, 7, 33, 17, 0, False, 127, 255, 7, "rand"),    # odd block
    (8, 8, 64, 64, 0, False, 64, 200, 3, "flat"),      # ties everywhere
    (16, 16, 40, 20, 1, False, 96, 300, 2, "sat"),
    (64, 64, 640, 400, 0, False, 64, 720, 1, "rand"),  # SadTest maximum area
    (1, 1, 5, 3, 0, False, 1, 16, 0, "rand"),
    (128, 4, 9, 2, 0, False, 128, 160, 3, "rand"),
]

NXM = [(w, h, ss, rs, off, kind) for (w, h, ss, rs, off, kind) in [
    (64, 32, 128, 256, 0, "rand"), (1, 1, 1, 1, 0, "rand"), (7, 5, 127, 129, 3, "rand"), (128, 64, 128, 131, 1, "sat"),
    (33, 17, 64, 127, 2, "rand"), (16, 16, 16, 16, 0, "flat"), (100, 3, 127, 200, 1, "rand"), (8, 64, 8, 8, 0, "rand"),
]]

EXT8 = [(sub, ss, rs, off, seed) for sub in (False, True) for (ss, rs, off, seed) in
        [(64, 64, 0, 1), (127, 131, 3, 2), (16, 16, 1, 3)]]
EXTALL = [(sub, ss, rs, off, seed) for sub in (False, True) for (ss, rs, off, seed) in
          [(64, 128, 0, 11), (127, 133, 1, 12), (64, 80, 3, 13)]]
DOWNSAMPLE = [(w, h, step) for (w, h, step) in [(64, 64, 2), (37, 21, 2), (128, 72, 4), (9, 9, 4), (3, 2, 2)]]
# svt_pme_sad_loop_kernel: (bw, bh, sa_w, sa_h, step, start_x, start_y, mvx, mvy, cost_type, src_stride,
# ref_stride, content, error_per_bit, initial best cost)
PME = [
    (8, 8, 16, 12, 1, -8, -6, 24, -40, 0, 64, 160, "rand", 100, 0xFFFFFFFF),   # entropy rate
    (16, 16, 30, 9, 2, -15, -4, 0, 0, 1, 127, 131, "rand", 60, 0xFFFFFFFF),    # L1 low-res, step 2, ragged width
    (32, 32, 24, 16, 3, -12, -8, -100, 56, 3, 96, 200, "rand", 80, 0xFFFFFFFF),  # L1 HD, step 3
    (64, 64, 17, 5, 1, -8, -2, 8, 8, 4, 64, 160, "rand", 1000, 0xFFFFFFFF),    # OPT
    (8, 4, 7, 3, 1, -3, -1, 0, 0, 0, 8, 24, "rand", 90, 0xFFFFFFFF),           # width < 8: nothing visited
    (4, 4, 40, 6, 2, -20, -3, 16, -16, 5, 16, 64, "flat", 0, 0xFFFFFFFF),      # no rate, ties: first minimum
    (128, 64, 12, 4, 1, -6, -2, -8, 24, 2, 128, 160, "rand", 70, 0xFFFFFFFF),  # mid-res lambda 0
    (16, 8, 33, 17, 2, -16, -8, 40, -8, 0, 32, 80, "sat", 200, 0xFFFFFFFF),    # saturated, entropy
    (8, 8, 24, 8, 1, -12, -4, 0, 0, 0, 64, 64, "flat", 50, 1),                  # initial best beats all
    # far reference MVs (ref_mv row, col): the MV difference wraps in the int16 MV of
    # mcomp.c:46 and |-32768| stays -32768 in abs_diff (mcomp.c:47)
    (8, 8, 16, 6, 1, -8, 0, 20000, -2768, 3, 64, 160, "rand", 80, 0xFFFFFFFF, (30000, -30000)),  # L1 HD
    (8, 8, 16, 6, 1, -8, 0, 20000, -2768, 0, 64, 160, "rand", 80, 0xFFFFFFFF, (30000, -30000)),  # entropy
    (16, 8, 20, 5, 2, -10, -2, -16000, 16000, 4, 64, 160, "rand", 40, 0xFFFFFFFF, (17000, -17000)),  # OPT
]


def _mv(rng):
    x = int(rng.integers(-300, 300))
    y = int(rng.integers(-200, 200))
    return ((y & 0xFFFF) << 16) | (x & 0xFFFF)


def _bests(rng, n, kind="mixed"):
    # a mix of MAX_SAD_VALUE and small values so both update branches run
    b = rng.integers(0, 60000, n).astype(np.uint32)
    b[rng.random(n) < 0.5] = 128 * 128 * 255
    return b


# ----------------------------------------------------------------------------
# runners
# ----------------------------------------------------------------------------
def _fn(lib, prefix, name):
    if prefix == "svt_":
        names = {"sad_loop_kernel": "svt_sad_loop_kernel_hip", "nxm_sad_kernel": "svt_nxm_sad_kernel_hip",
                 "sad_16b_kernel": "svt_aom_sad_16b_kernel_hip", "downsample_2d": "svt_aom_downsample_2d_hip",
                 "initialize_buffer_32bits": "svt_initialize_buffer_32bits_hip",
                 "pme_sad_loop_kernel": "svt_pme_sad_loop_kernel_hip"}
        return getattr(lib, names.get(name, "svt_" + name + "_hip"))
    return getattr(lib, prefix + name)


def run_sad_loop(lib, prefix, case, seed):
    bw, bh, sa_w, sa_h, skip, sub, ss, raw, off, kind = case
    rng = np.random.default_rng(seed)
    src = _content(rng, (2 * ss if sub else ss) * bh + bw + 16, kind)
    rstride = 2 * raw if sub else raw
    n = off + (sa_h - 1) * raw + (bh - 1) * rstride + sa_w + bw + 16
    ref = _content(rng, n, kind)
    best = C.c_uint64(0)
    x = C.c_int16(-7)
    y = C.c_int16(-9)
    f = _fn(lib, prefix, "sad_loop_kernel")
    f.restype = None
    f(_u8(src), C.c_uint32(2 * ss if sub else ss), C.cast(C.c_void_p(ref.ctypes.data + off), U8P),
      C.c_uint32(rstride), C.c_uint32(bh), C.c_uint32(bw), C.byref(best), C.byref(x), C.byref(y), C.c_uint32(raw),
      C.c_uint8(skip), C.c_int16(sa_w), C.c_int16(sa_h))
    return {"best": np.array([best.value], np.uint64), "xy": np.array([x.value, y.value], np.int16)}


def run_nxm(lib, prefix, case, seed, bits16=False):
    w, h, ss, rs, off, kind = case
    rng = np.random.default_rng(seed)
    if bits16:
        src = _content(rng, ss * h + w + 8, kind, 1024, np.uint16)
        ref = _content(rng, off + rs * h + w + 8, kind, 1024, np.uint16)
        f = _fn(lib, prefix, "sad_16b_kernel")
        f.restype = C.c_uint32
        v = f(src.ctypes.data_as(U16P), C.c_uint32(ss), C.cast(C.c_void_p(ref.ctypes.data + 2 * off), U16P),
              C.c_uint32(rs), C.c_uint32(h), C.c_uint32(w))
    else:
        src = _content(rng, ss * h + w + 8, kind)
        ref = _content(rng, off + rs * h + w + 8, kind)
        f = _fn(lib, prefix, "nxm_sad_kernel")
        f.restype = C.c_uint32
        v = f(_u8(src), C.c_uint32(ss), C.cast(C.c_void_p(ref.ctypes.data + off), U8P), C.c_uint32(rs),
              C.c_uint32(h), C.c_uint32(w))
    return {"sad": np.array([v], np.uint32)}


def run_ext8(lib, prefix, case):
    sub, ss, rs, off, seed = case
    rng = np.random.default_rng(seed)
    src = _content(rng, ss * 16 + 32, "rand")
    ref = _content(rng, off + rs * 16 + 32, "rand")
    b8, b16 = _bests(rng, 4), _bests(rng, 1)
    m8, m16 = rng.integers(0, 2**32, 4, dtype=np.uint64).astype(np.uint32), np.zeros(1, np.uint32)
    s16, s8 = np.zeros(1, np.uint32), np.zeros(4, np.uint32)
    mv = _mv(rng)
    f = _fn(lib, prefix, "ext_sad_calculation_8x8_16x16")
    f.restype = None
    f(_u8(src), C.c_uint32(ss), C.cast(C.c_void_p(ref.ctypes.data + off), U8P), C.c_uint32(rs), _u32(b8), _u32(b16),
      _u32(m8), _u32(m16), C.c_uint32(mv), _u32(s16), _u32(s8), C.c_bool(sub))
    return {"b8": b8, "b16": b16, "m8": m8, "m16": m16, "s16": s16, "s8": s8}


def run_ext32(lib, prefix, seed):
    rng = np.random.default_rng(seed)
    s16 = rng.integers(0, 30000, 16).astype(np.uint32)
    b32, b64 = _bests(rng, 4) * 4, _bests(rng, 1) * 16
    m32, m64 = np.zeros(4, np.uint32), np.zeros(1, np.uint32)
    s32 = np.zeros(4, np.uint32)
    f = _fn(lib, prefix, "ext_sad_calculation_32x32_64x64")
    f.restype = None
    f(_u32(s16), _u32(b32), _u32(b64), _u32(m32), _u32(m64), C.c_uint32(_mv(rng)), _u32(s32))
    return {"b32": b32, "b64": b64, "m32": m32, "m64": m64, "s32": s32}


def run_extall(lib, prefix, case):
    sub, ss, rs, off, seed = case
    rng = np.random.default_rng(seed)
    src = _content(rng, ss * 64 + 64, "rand")
    ref = _content(rng, off + rs * 64 + 80, "rand")
    b8, b16 = _bests(rng, 64), _bests(rng, 16)
    m8, m16 = np.zeros(64, np.uint32), np.zeros(16, np.uint32)
    e16 = np.zeros((16, 8), np.uint32)
    e8 = np.zeros((64, 8), np.uint32)
    f = _fn(lib, prefix, "ext_all_sad_calculation_8x8_16x16")
    f.restype = None
    f(_u8(src), C.c_uint32(ss), C.cast(C.c_void_p(ref.ctypes.data + off), U8P), C.c_uint32(rs),
      C.c_uint32(_mv(rng)), _u32(b8), _u32(b16), _u32(m8), _u32(m16), _u32(e16), _u32(e8), C.c_bool(sub))
    return {"b8": b8, "b16": b16, "m8": m8, "m16": m16, "e16": e16}  # e8 is not written by the C reference


def run_ext_eight32(lib, prefix, seed):
    rng = np.random.default_rng(seed)
    s16 = rng.integers(0, 30000, (16, 8)).astype(np.uint32)
    b32, b64 = _bests(rng, 4) * 4, _bests(rng, 1) * 16
    m32, m64 = np.zeros(4, np.uint32), np.zeros(1, np.uint32)
    s32 = np.zeros((4, 8), np.uint32)
    f = _fn(lib, prefix, "ext_eight_sad_calculation_32x32_64x64")
    f.restype = None
    f(_u32(s16), _u32(b32), _u32(b64), _u32(m32), _u32(m64), C.c_uint32(_mv(rng)), _u32(s32))
    return {"b32": b32, "b64": b64, "m32": m32, "m64": m64, "s32": s32}


def run_init(lib, prefix, c128, c32, value):
    buf = np.full(c128 * 4 + c32 + 5, 0xA5A5A5A5, np.uint32)
    f = _fn(lib, prefix, "initialize_buffer_32bits")
    f.restype = None
    f(_u32(buf), C.c_uint32(c128), C.c_uint32(c32), C.c_uint32(value))
    return {"buf": buf}


def run_downsample(lib, prefix, case, seed):
    w, h, step = case
    rng = np.random.default_rng(seed)
    stride = w + 5
    inp = rng.integers(0, 256, stride * (h + 1), dtype=np.int64).astype(np.uint8)
    ostride = w // step + 3
    out = np.full(ostride * (h // step + 2), 0x5A, np.uint8)
    f = _fn(lib, prefix, "downsample_2d")
    f.restype = None
    f(_u8(inp), C.c_uint32(stride), C.c_uint32(w), C.c_uint32(h), _u8(out), C.c_uint32(ostride), C.c_uint32(step))
    return {"out": out}


class MvCostParams(C.Structure):
    """MV_COST_PARAMS (reference mcomp.h:37-48)."""
    _fields_ = [("ref_mv", C.POINTER(C.c_int16)), ("full_ref_mv", C.c_int16 * 2), ("mv_cost_type", C.c_uint8),
                ("mvjcost", C.POINTER(C.c_int)), ("mvcost", C.POINTER(C.c_int) * 2), ("error_per_bit", C.c_int),
                ("early_exit_th", C.c_int), ("sad_per_bit", C.c_int)]


def run_pme(lib, prefix, case, seed):
    bw, bh, sa_w, sa_h, step, sx, sy, mvx, mvy, ctype, ss, rs, kind, epb, best0 = case[:15]
    rng = np.random.default_rng(seed)
    src = _content(rng, ss * bh + bw + 16, kind)
    ref = _content(rng, rs * (sa_h + bh + 1) + sa_w + bw + 16, kind)
    ref_mv = np.array([int(rng.integers(-64, 64)), int(rng.integers(-64, 64))], np.int16)
    if len(case) > 15:
        ref_mv = np.array(case[15], np.int16)
    jc = rng.integers(100, 2000, 4).astype(np.int32)
    tabs = [rng.integers(0, 4000, 2 * 16384 + 1).astype(np.int32) for _ in range(2)]
    p = MvCostParams()
    p.ref_mv = ref_mv.ctypes.data_as(C.POINTER(C.c_int16))
    p.mv_cost_type = ctype
    p.mvjcost = jc.ctypes.data_as(C.POINTER(C.c_int))
    for k in range(2):
        p.mvcost[k] = C.cast(C.c_void_p(tabs[k].ctypes.data + 4 * 16384), C.POINTER(C.c_int))
    p.error_per_bit = epb
    best = C.c_uint32(best0)
    bx, by = C.c_int16(-5), C.c_int16(-7)
    f = _fn(lib, prefix, "pme_sad_loop_kernel")
    f.restype = None
    f(C.byref(p), _u8(src), C.c_uint32(ss), _u8(ref), C.c_uint32(rs), C.c_uint32(bh), C.c_uint32(bw), C.byref(best),
      C.byref(bx), C.byref(by), C.c_int16(sx), C.c_int16(sy), C.c_int16(sa_w), C.c_int16(sa_h), C.c_int16(step),
      C.c_int16(mvx), C.c_int16(mvy))
    return {"cost": np.array([best.value], np.uint32), "mv": np.array([bx.value, by.value], np.int16)}


def all_cases():
    """(name, callable(lib, prefix) -> dict) for every case."""
    cases = []
    for i, c in enumerate(SAD_LOOP):
        cases.append((f"sad_loop_{i}", lambda lib, p, c=c, i=i: run_sad_loop(lib, p, c, 100 + i)))
    for i, c in enumerate(NXM):
        cases.append((f"nxm_{i}", lambda lib, p, c=c, i=i: run_nxm(lib, p, c, 200 + i)))
        cases.append((f"sad16b_{i}", lambda lib, p, c=c, i=i: run_nxm(lib, p, c, 300 + i, bits16=True)))
    for i, c in enumerate(EXT8):
        cases.append((f"ext8x8_16x16_{i}", lambda lib, p, c=c: run_ext8(lib, p, c)))
    for i in range(4):
        cases.append((f"ext32x32_64x64_{i}", lambda lib, p, i=i: run_ext32(lib, p, 400 + i)))
    for i, c in enumerate(EXTALL):
        cases.append((f"ext_all_{i}", lambda lib, p, c=c: run_extall(lib, p, c)))
    for i in range(4):
        cases.append((f"ext_eight32_{i}", lambda lib, p, i=i: run_ext_eight32(lib, p, 500 + i)))
    for i, (a, b, v) in enumerate([(21, 1, 128 * 128 * 255), (0, 3, 7), (1, 0, 0)]):
        cases.append((f"init32_{i}", lambda lib, p, a=a, b=b, v=v: run_init(lib, p, a, b, v)))
    for i, c in enumerate(DOWNSAMPLE):
        cases.append((f"downsample_{i}", lambda lib, p, c=c, i=i: run_downsample(lib, p, c, 600 + i)))
    for i, c in enumerate(PME):
        cases.append((f"pme_{i}", lambda lib, p, c=c, i=i: run_pme(lib, p, c, 700 + i)))
    return cases
