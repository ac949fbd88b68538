"""Average rocprofv3 PMC counters per k_me_sb launch from gpurun_out/pmc_*/ CSVs.

FETCH_SIZE / WRITE_SIZE are KB; FETCH_SIZE is doubled for gfx950
(MI355X_MICROARCH.md, HBM section: FETCH_SIZE reports half the bytes of wide
coalesced reads). Writes profiles-ready JSON to <out>/pmc_summary.json.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(out):
    per = defaultdict(list)
    for path in glob.glob(os.path.join(out, "pmc_*", "**", "*counter_collection.csv"), recursive=True):
        with open(path) as fh:
            rows = list(csv.DictReader(fh))
        by_dispatch = defaultdict(dict)
        for r in rows:
            if "k_me_sb" not in r["Kernel_Name"]:
                continue
            by_dispatch[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
        for d in by_dispatch.values():
            for k, v in d.items():
                per[k].append(v)
    avg = {k: sum(v) / len(v) for k, v in per.items() if v}
    res = {"counters_avg_per_launch": avg}
    if "FETCH_SIZE" in avg:
        res["fetch_bytes_corrected"] = avg["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in avg:
        res["write_bytes"] = avg["WRITE_SIZE"] * 1024
    if "fetch_bytes_corrected" in res and "write_bytes" in res:
        res["hbm_bytes_per_launch"] = res["fetch_bytes_corrected"] + res["write_bytes"]
    print(json.dumps(res, indent=1))
    with open(os.path.join(out, "pmc_summary.json"), "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
