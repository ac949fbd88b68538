"""profiles/<tag>/phases.json from one GPU session's phase measurements.

inputs: the stdout of scripts/gpu_phase_cost.sh (phase_cost.py lines, 4
pictures per launch) and the rocprofv3 CSVs of scripts/gpu_phase_pmc.sh (one
picture per launch), both over the stop-after builds KS (scripts/
build_phase_libs.sh). A phase's cost is the difference between consecutive
builds; VALU busy = SQ_ACTIVE_INST_VALU quad-cycles x 4 / 1024 SIMDs / clock.

usage: python3 scripts/phases_json.py <phase_cost.log> <phase_pmc dir> <out.json>
"""
import csv
import glob
import json
import os
import re
import sys

KS = ["1", "2", "3", "4", "5", "55", "6", "full"]
NAMES = ["start..A0", "A1 table", "A1 tiles", "D + L1 table", "L1 tiles", "final centre", "full-pel",
         "decode, records, candidates"]
CLOCK_GHZ = 2.15  # SQ_BUSY_CYCLES / wall of the same passes (MI355X under this load)


def main():
    log, pmc_dir, out = sys.argv[1:4]
    cost = {}
    for line in open(log):
        m = re.search(r"stop_after_(\w+)\s+\S+ x(\d+):\s+([\d.]+) us per launch,\s+([\d.]+) us per picture", line)
        if m:
            cost[m.group(1)] = float(m.group(4))
    ctr = {}
    for k in KS:
        f = glob.glob(os.path.join(pmc_dir, f"stop{k}", "**", "*counter_collection.csv"), recursive=True)
        acc, disp = {}, set()
        for r in csv.DictReader(open(f[0])) if f else []:
            acc[r["Counter_Name"]] = acc.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            disp.add(r["Dispatch_Id"])
        ctr[k] = {c: v / max(1, len(disp)) for c, v in acc.items()}
    phases, pc, pk = [], 0.0, {}
    for k, name in zip(KS, NAMES):
        c = cost.get(k)
        e = {"phase": name, "cost_us_per_picture_x4": None if c is None else round(c - pc, 2)}
        if ctr[k]:
            d = {n: ctr[k][n] - pk.get(n, 0.0) for n in ctr[k]}
            e["valu_busy_us_per_simd_x1"] = round(d.get("SQ_ACTIVE_INST_VALU", 0) * 4 / 1024 / (CLOCK_GHZ * 1e3), 2)
            for n in ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD"):
                if n in d:
                    e[n] = int(round(d[n]))
            pk = ctr[k]
        if c is not None:
            pc = c
        phases.append(e)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import kernel_code_sha

    res = {"workload": "4k_p8", "code_sha": kernel_code_sha(),
           "note": "phase costs: differences between SVTME_STOP_AFTER=k builds (scripts/gpu_phase_cost.sh, 4 "
                   "pictures per launch, us per picture); counters: same builds, one picture per launch "
                   "(scripts/gpu_phase_pmc.sh, per launch); VALU busy = SQ_ACTIVE_INST_VALU quad-cycles x 4 / "
                   f"1024 SIMDs / {CLOCK_GHZ} GHz",
           "phases": phases,
           "total_us_per_picture_x4": cost.get("full")}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
