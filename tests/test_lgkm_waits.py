"""k_fp_wide's inline-asm LDS reads: in the machine code of
the built library, no instruction touches a VGPR an LDS / scalar-memory load
may still be writing (tests/lgkm_check.py: a control-flow may-analysis of
s_waitcnt lgkmcnt over every kernel). A second case removes each of
k_fp_wide's lgkmcnt(k > 0) waits in turn and requires the check to flag it,
so the analysis is known to see the inline reads."""
import os
import shutil

import pytest

import lgkm_check as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "svt-av1-mirror_amd", "libsvtme.so")

pytestmark = pytest.mark.skipif(
    not (os.path.exists(LIB) and shutil.which("objcopy") and os.path.exists(f"{L.LLVM}/llvm-objdump")),
    reason="needs the built libsvtme.so, objcopy and the ROCm llvm tools")


@pytest.fixture(scope="module")
def kernels(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("co"))
    funcs = {}
    for co in L.code_objects(LIB, d):
        funcs.update(L.functions(L.disassemble(co)))
    assert any("k_fp_wide" in name for name in funcs), "k_fp_wide not found in the library's code objects"
    return funcs


def test_no_lgkm_result_used_before_its_wait(kernels):
    bad = {name: v[:5] for name, ins in kernels.items() if (v := L.check(ins))}
    assert not bad, bad


def test_check_flags_a_removed_wait(kernels):
    name = next(n for n in kernels if "k_fp_wide" in n)
    ins = kernels[name]
    waits = [i for i, (_, t) in enumerate(ins)
             if t.startswith("s_waitcnt") and "lgkmcnt(" in t and "lgkmcnt(0)" not in t]
    assert len(waits) >= 8, "k_fp_wide has no partial lgkmcnt waits: the inline reads are gone?"
    for i in waits:
        mutant = ins[:i] + [(ins[i][0], "s_nop 0")] + ins[i + 1:]
        assert L.check(mutant), f"removing the wait at +{ins[i][0]:#x} went unnoticed"
