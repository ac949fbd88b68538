"""Per-phase instruction counts from scripts/gpu_phase_pmc.sh output (average per k_hme launch)."""
import csv
import glob
import os
import sys

O = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/phase_pmc"
NAMES = ["start..A0", "A1 table", "A1 tiles", "D + L1 table", "L1 tiles", "full-pel", "decode+tail"]
rows = []
for k in ["1", "2", "3", "4", "5", "6", "full"]:
    f = glob.glob(os.path.join(O, f"stop{k}", "**", "*counter_collection.csv"), recursive=True)
    if not f:
        print("missing", k)
        sys.exit(1)
    acc, disp = {}, set()
    for r in csv.DictReader(open(f[0])):
        acc[r["Counter_Name"]] = acc.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        disp.add(r["Dispatch_Id"])
    n = max(1, len(disp))
    rows.append({c: v / n for c, v in acc.items()})
cs = sorted(rows[0])
print(f"{'phase':16s}" + "".join(f"{c:>22s}" for c in cs))
prev = {c: 0.0 for c in cs}
for name, r in zip(NAMES, rows):
    print(f"{name:16s}" + "".join(f"{r[c] - prev[c]:22.0f}" for c in cs))
    prev = r
print(f"{'total':16s}" + "".join(f"{rows[-1][c]:22.0f}" for c in cs))
