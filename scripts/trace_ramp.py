"""Per-launch durations of one kernel over a process's life, from a rocprofv3
--kernel-trace CSV: mean duration and start-to-start gap per block of N launches.

usage: python3 scripts/trace_ramp.py TRACE.csv [kernel_prefix=void svtme::k_hme] [block=20]
"""
import csv
import json
import sys

import numpy as np


def main():
    path = sys.argv[1]
    pref = sys.argv[2] if len(sys.argv) > 2 else "void svtme::k_hme"
    blk = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    rows = [r for r in csv.DictReader(open(path)) if r["Kernel_Name"].startswith(pref)]
    s = np.array([int(r["Start_Timestamp"]) for r in rows], np.int64)
    e = np.array([int(r["End_Timestamp"]) for r in rows], np.int64)
    o = np.argsort(s)
    s, e = s[o], e[o]
    d = (e - s) / 1e3
    gap = np.diff(s) / 1e3
    print(json.dumps({"kernel": rows[0]["Kernel_Name"] if rows else pref, "launches": len(rows), "block": blk,
                      "duration_us_per_block": [round(float(d[i:i + blk].mean()), 2) for i in range(0, len(d), blk)],
                      "start_gap_us_per_block": [round(float(gap[i:i + blk].mean()), 2)
                                                 for i in range(0, len(gap), blk)],
                      "t_ms_at_block_start": [round(float((s[i] - s[0]) / 1e6), 3) for i in range(0, len(s), blk)]}))


if __name__ == "__main__":
    main()
