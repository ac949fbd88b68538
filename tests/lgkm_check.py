"""Static check of LDS / scalar-memory result use in a gfx950 disassembly.

k_fp_wide issues its LDS row reads as inline-asm `ds_read_b64` with explicit
`s_waitcnt lgkmcnt(k)` (svtme_stages.hip, fpw_row_issue / fpw_row_wait), so
the compiler does not know those registers are in flight: a register copy or
spill of a destination before its wait would read stale data. This module
walks the machine code of a kernel (llvm-objdump output) over its control-flow
graph and reports every instruction that reads or writes a VGPR an LGKM load
may still be writing.

Model: every LGKM instruction (ds_*, s_load*, s_buffer_load*, s_memtime,
s_memrealtime, s_sendmsg*) enters a queue entry (its destination VGPRs, if it
is a VGPR load); `s_waitcnt lgkmcnt(k)` retires the entries with at least k
younger LGKM instructions, unless a scalar-memory load (which may return out of
order) is younger than the entry, in which case only lgkmcnt(0) retires it.
Join points take the union of entries (the youngest age of each). The
analysis is a forward may-analysis iterated to a fixed point, so it is
conservative: it may flag a use the hardware would in fact order, never the
reverse.

Test infrastructure (tests/test_lgkm_waits.py); not part of the product.
"""
import re
import subprocess

LLVM = "/opt/rocm/lib/llvm/bin"
_VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
_TARGET = re.compile(r"<[^>+]+\+0x([0-9a-f]+)>")
_LGKM_WAIT = re.compile(r"lgkmcnt\((\d+)\)")
MAX_AGE = 64


def code_objects(lib_path, workdir):
    """Device code objects (gfx950) embedded in a HIP shared library."""
    import os

    fb = os.path.join(workdir, "fatbin.bin")
    # (an explicit output file: objcopy with none rewrites its input in place, and the
    # library may be mapped by the running process)
    subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fb}", lib_path, os.path.join(workdir, "scratch.so")],
                   check=True)
    data = open(fb, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    offs, i = [], data.find(magic)
    while i >= 0:
        offs.append(i)
        i = data.find(magic, i + 1)
    out = []
    for k, o in enumerate(offs):
        e = offs[k + 1] if k + 1 < len(offs) else len(data)
        b = os.path.join(workdir, f"b{k}.bin")
        co = os.path.join(workdir, f"co{k}.o")
        with open(b, "wb") as fh:
            fh.write(data[o:e])
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={b}", f"--output={co}"],
                           capture_output=True)
        if r.returncode == 0 and os.path.getsize(co) > 0:
            out.append(co)
    return out


def disassemble(co):
    r = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], capture_output=True, text=True,
                       check=True)
    return r.stdout


def functions(dis):
    """{symbol: [(offset, text)]} of a disassembly."""
    funcs, cur, base = {}, None, 0
    for line in dis.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.+)>:$", line)
        if m:
            cur, base = m.group(2), int(m.group(1), 16)
            funcs[cur] = []
            continue
        if cur is None:
            continue
        m = re.match(r"^\s+(\S.*?)\s*//\s*([0-9A-F]+):", line)
        if m:
            t = _TARGET.search(line)  # a branch's target, after the encoding comment
            funcs[cur].append((int(m.group(2), 16) - base, m.group(1) + (" " + t.group(0) if t else "")))
    return funcs


def vregs(operands):
    regs = set()
    for m in _VREG.finditer(operands):
        if m.group(3) is not None:
            regs.add(int(m.group(3)))
        else:
            regs.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return regs


def _kind(op):
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("s_load", "s_buffer_load", "s_memtime", "s_memrealtime", "s_sendmsg", "s_dcache")):
        return "smem"
    return None


def check(insts):
    """Violations [(offset, instruction, pending VGPRs it touches, offset of the load)]."""
    n = len(insts)
    index = {off: i for i, (off, _) in enumerate(insts)}
    succ = []
    for i, (off, text) in enumerate(insts):
        op = text.split()[0]
        s = []
        t = _TARGET.search(text)
        if op.startswith("s_cbranch") or op == "s_branch":
            if t and int(t.group(1), 16) in index:
                s.append(index[int(t.group(1), 16)])
            if op != "s_branch" and i + 1 < n:
                s.append(i + 1)
        elif op in ("s_endpgm", "s_setpc_b64", "s_trap"):
            pass
        elif i + 1 < n:
            s.append(i + 1)
        succ.append(s)
    # state: {load offset: (frozenset dst vgprs, age, smem_younger)}
    states = [None] * n
    states[0] = {}
    work = [0]
    viol = {}
    while work:
        i = work.pop()
        st = dict(states[i])
        off, text = insts[i]
        parts = text.split(None, 1)
        op, operands = parts[0], parts[1] if len(parts) > 1 else ""
        kind = _kind(op)
        regs = vregs(operands)
        # a touch of a pending destination (the LGKM instruction's own address
        # operands included; its destination is checked as a write-after-write)
        for lo, (dst, age, sy) in st.items():
            hit = regs & dst
            if hit and lo != off:
                viol[(off, lo)] = (off, text, sorted(hit), lo)
        if op == "s_waitcnt":
            m = _LGKM_WAIT.search(operands)
            if m:
                k = int(m.group(1))
                st = {lo: e for lo, e in st.items() if not (k == 0 or (e[1] >= k and not e[2]))}
        if kind:
            st = {lo: (d, min(MAX_AGE, a + 1), sy or kind == "smem") for lo, (d, a, sy) in st.items()}
            dst = set()
            if kind == "lds" and ("read" in op or "load" in op or "bpermute" in op or "permute" in op
                                  or "swizzle" in op or "_rtn" in op):
                first = operands.split(",")[0]
                dst = vregs(first)
            st[off] = (frozenset(dst), 0, False)
        for j in succ[i]:
            old = states[j]
            if old is None:
                new = st
            else:
                new = dict(old)
                for lo, (d, a, sy) in st.items():
                    if lo in new:
                        od, oa, osy = new[lo]
                        new[lo] = (d, min(a, oa), sy or osy)
                    else:
                        new[lo] = (d, a, sy)
            if new != old:
                states[j] = new
                work.append(j)
    return sorted(viol.values())
