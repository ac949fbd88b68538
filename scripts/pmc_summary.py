"""Average rocprofv3 PMC counters per ME-pass launch from <out>/pmc_*/ CSVs.

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

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import kernel_code_sha  # noqa: E402


def main(out):
    per = defaultdict(list)
    per_kernel = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(os.path.join(out, "pmc_*", "**", "*counter_collection.csv"), recursive=True):
        with open(path) as fh:
            rows = list(csv.DictReader(fh))
        by_dispatch = defaultdict(dict)
        names = {}
        for r in rows:
            if not any(t in r["Kernel_Name"] for t in ("k_stage", "k_hme", "k_fp", "k_l0", "k_l1")):
                continue
            by_dispatch[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"].split("(")[0]
        for disp, d in by_dispatch.items():
            for k, v in d.items():
                per_kernel[names[disp]][k].append(v)
    kern = {n: {k: sum(v) / len(v) for k, v in d.items() if v} for n, d in per_kernel.items()}
    # one "launch" of the ME path = one dispatch of every stage kernel
    avg = defaultdict(float)
    for d in kern.values():
        for k, v in d.items():
            avg[k] += v
    res = {"counters_avg_per_launch": dict(avg), "per_kernel": kern}
    for k, d in kern.items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_bytes"] = d["FETCH_SIZE"] * 1024 * 2 + d["WRITE_SIZE"] * 1024
    try:  # the launch size the counters belong to (bench.json of the same profile)
        with open(os.path.join(out, "bench.json")) as fh:
            b = json.loads(fh.read().strip().splitlines()[-1])
        res["sbs_per_launch"] = b["roofline"]["sbs_per_launch"]
        res["workload"] = b["config"].get("name")
    except (OSError, ValueError, KeyError, IndexError):
        pass
    res["code_sha"] = kernel_code_sha()  # the stage sources these counters were taken on
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
