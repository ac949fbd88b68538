"""The ME rate the encoder gets through the glue (integration/svtme_svt_glue.c):
whole encodes with svtav1enc_gpu (SVTME_GLUE_STRICT, no pyramid verification,
which would download every pyramid), their bitstreams checked against the
unmodified reference encoder, and the glue's exit stats: served_sb_per_s = SBs
of the GPU jobs / the wall time with at least one job in flight (upload,
search and the packed copy back included), mean job latency, jobs in flight.

usage: python scripts/glue_rate.py OUT.json [case ...]   (default: 4k_p8_64f 4k_p8_16f 1080p_p8)
(environment: SVTME_GLUE_* of integration/svtme_svt_glue.c pass through, e.g.
SVTME_GLUE_PIN=0 for uploads through the library's staging ring)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "svt-av1-mirror_amd"))

import encoder_harness as E  # noqa: E402


def main():
    out = sys.argv[1]
    cases = sys.argv[2:] or ["4k_p8_64f", "4k_p8_16f", "1080p_p8"]
    wd = os.path.join("/tmp", "svtme_glue_rate")
    res = []
    reps = int(os.environ.get("GLUE_RATE_REPEAT", "1"))  # the same encode several times (a rare stall's odds)
    refs = {}
    for case in [c for c in cases for _ in range(reps)]:
        ref = refs.get(case) or E.encode("ref", case, wd)
        refs[case] = ref
        trace = os.path.join(wd, f"{case}.trace.jsonl")
        got = E.encode("gpu", case, wd, env_extra={"SVTME_GLUE_VERIFY": "0", "SVTME_GLUE_TRACE": trace})
        g = got["glue"]
        with open(trace) as fh:
            lines = [json.loads(line) for line in fh if line.strip()]
        jobs = [t for t in lines if t["tf"] < 2]
        ups = [t for t in lines if t["tf"] == 2]  # uploads (start create_ms, end done_ms)
        regs = [t for t in lines if t["tf"] == 3]  # page-lockings of encoder buffers (hipHostRegister)
        w, h, frames, preset = E.CASES[case][:4]
        r = {"case": case, "size": f"{w}x{h}", "frames": frames, "preset": preset,
             "identical": got["md5"] == ref["md5"], "md5": got["md5"], "ref_seconds": ref["seconds"],
             "gpu_encoder_seconds": got["seconds"], **g, "svtme_log": got.get("svtme_log", []),
             "jobs": jobs, "uploads_trace": ups,
             "registrations_trace": regs}
        lat = sorted(j["done_ms"] - j["create_ms"] for j in jobs)
        # jobs above 1 ms and the uploads that overlapped them (a stall's candidates)
        r["long_jobs"] = [{"pn": j["pn"], "tf": j["tf"], "ms": round(j["done_ms"] - j["create_ms"], 3),
                           "gpu_ms": j.get("gpu_ms"), "copy_ms": j.get("copy_ms"),
                           "uploads_overlapping": [u["pn"] for u in ups
                                                   if u["create_ms"] < j["done_ms"] and u["done_ms"] > j["create_ms"]],
                           "registrations_overlapping": [round(u["done_ms"] - u["create_ms"], 3) for u in regs
                                                         if u["create_ms"] < j["done_ms"] and u["done_ms"] > j["create_ms"]]}
                          for j in jobs if j["done_ms"] - j["create_ms"] > 1.0]
        r["max_job_ms"] = round(lat[-1], 3)
        ud = sorted(u["done_ms"] - u["create_ms"] for u in ups)  # each upload call on an analysis thread
        if ud:
            r["upload_call_ms"] = {"median": round(ud[len(ud) // 2], 4), "max": round(ud[-1], 3),
                                   "mean": round(sum(ud) / len(ud), 4), "over_1ms": sum(d > 1.0 for d in ud)}
        print(json.dumps({k: v for k, v in r.items() if k not in ("jobs", "uploads_trace", "registrations_trace")}),
              flush=True)
        print(f"  job latency ms: min {lat[0]:.3f} median {lat[len(lat) // 2]:.3f} max {lat[-1]:.3f}; "
              f"submit part median {sorted(j['submitted_ms'] - j['create_ms'] for j in jobs)[len(jobs) // 2]:.3f}",
              flush=True)
        res.append(r)
        if not r["identical"]:
            raise SystemExit(f"{case}: bitstream differs from the reference encoder")
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
