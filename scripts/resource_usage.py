"""Per-kernel resource usage of a HIP source for gfx950 (container, no GPU):
VGPRs, SGPRs, spills, scratch, LDS and occupancy from the compiler's
kernel-resource-usage remarks.
usage: python scripts/resource_usage.py [source.hip] [name-regex] [-- extra hipcc flags]"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def usage(src, extra=()):
    src = os.path.abspath(src)
    with tempfile.TemporaryDirectory() as td:
        r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c",
                            "-o", os.path.join(td, "k.o"), src, "-Rpass-analysis=kernel-resource-usage", *extra],
                           capture_output=True, text=True, cwd=td)
    if r.returncode:
        raise SystemExit(r.stderr[-3000:])
    out, cur = {}, None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: ([^:]+): (.*?) \[-Rpass", line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2).strip()
        if k == "Function Name":
            cur = v
            out[cur] = {}
        elif cur:
            out[cur][k] = v
    return out


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.splitlines()


if __name__ == "__main__":
    args = sys.argv[1:]
    extra = []
    if "--" in args:
        extra = args[args.index("--") + 1:]
        args = args[:args.index("--")]
    src = args[0] if args and args[0] else os.path.join(ROOT, "svt-av1-mirror_amd", "csrc", "svtme_stages.hip")
    pat = re.compile(args[1] if len(args) > 1 else ".")
    u = usage(src, extra)
    names = list(u)
    for n, d in zip(names, demangle(names)):
        if not pat.search(d):
            continue
        v = u[n]
        print(f"{d[:60]:60s} VGPR {v.get('VGPRs', '?'):>4} AGPR {v.get('AGPRs', '?'):>3} SGPR "
              f"{v.get('TotalSGPRs', '?'):>4} spillV {v.get('VGPRs Spill', '?'):>3} spillS "
              f"{v.get('SGPRs Spill', '?'):>3} scratch {v.get('ScratchSize [bytes/lane]', '?'):>4} "
              f"LDS {v.get('LDS Size [bytes/block]', '?'):>6} occ {v.get('Occupancy [waves/SIMD]', '?')}")
