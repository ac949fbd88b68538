"""Per-kernel rtcd parity (the `*_hip` drop-in variants and their checker).

Golden outputs in tests/golden/rtcd_cases.npz come from the reference's own
C kernels compiled from source (AVX2 agreeing on every case; see
tests/golden/make_golden.py). CPU: the oracle's kernel restatements
(oracle/svtme_oracle_kernels.c) equal them. GPU (-m gpu): the product's
`*_hip` variants equal them, bit-exact, including unaligned pointers, odd
strides, widths 1..128 and the 640 x 400 maximum search area.
"""
import ctypes as C
import os

import numpy as np
import pytest

import rtcd_cases as R
from conftest import PKG, ROOT

GOLD = np.load(os.path.join(ROOT, "tests", "golden", "rtcd_cases.npz"))
CASES = R.all_cases()


def _check(name, got):
    for k, v in got.items():
        exp = GOLD[f"{name}/{k}"]
        assert np.array_equal(np.asarray(v).reshape(exp.shape), exp), (name, k)


@pytest.mark.parametrize("name,run", CASES, ids=[c[0] for c in CASES])
def test_oracle_kernels_vs_golden(svtme, name, run):
    _check(name, run(svtme.load_oracle(), "svtora_"))


@pytest.mark.gpu
@pytest.mark.parametrize("name,run", CASES, ids=[c[0] for c in CASES])
def test_hip_kernels_vs_golden(svtme, name, run):
    lib = svtme.load_product()
    lib.svtme_rtcd_failed()  # clear this thread's flag
    _check(name, run(lib, "svt_"))
    assert lib.svtme_rtcd_failed() == 0, lib.svtme_last_error()


@pytest.mark.gpu
def test_hip_sad_loop_random_sweep(svtme):
    """Extra random shapes checked against the oracle (no golden needed)."""
    lib, ora = svtme.load_product(), svtme.load_oracle()
    rng = np.random.default_rng(77)
    for i in range(24):
        bw = int(rng.choice([4, 8, 12, 16, 24, 32, 48, 64]))
        bh = int(rng.integers(1, 33))
        sub = bool(rng.integers(0, 2))
        case = (bw, bh, int(rng.integers(1, 70)), int(rng.integers(1, 40)), int(rng.integers(0, 2)), sub,
                int(rng.integers(bw, bw + 70)), int(rng.integers(bw + 72, bw + 300)), int(rng.integers(0, 4)),
                str(rng.choice(["rand", "flat", "sat"])))
        a = R.run_sad_loop(lib, "svt_", case, 1000 + i)
        b = R.run_sad_loop(ora, "svtora_", case, 1000 + i)
        for k in a:
            assert np.array_equal(a[k], b[k]), (case, k, a, b)
