"""First-job latency in a fresh process: context creation, then the first,
second and third packed submission of a 4K TF-ME job (split path) and of a 4K
p8 PA-ME job (k_hme), each waited for. Prints milliseconds."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "svt-av1-mirror_amd"))

import svtme as S  # noqa: E402
import workloads as W  # noqa: E402


def main():
    out = {}
    t0 = time.perf_counter()
    gpu = S.GpuME(0)
    out["ctx_create_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
    for name in ("4k_tf_p8", "4k_p8"):
        for t, f in W.workload_frames(name).items():
            gpu.upload(t, f)
    gpu.sync()
    pa = S.PackLayout()
    pa.n_pus, pa.max_cand, pa.max_refs, pa.full_records, pa.sb_results = 85, 6, 3, 0, 1
    tf = S.PackLayout()
    tf.full_records = 1
    for name, L in (("4k_tf_p8", tf), ("4k_p8", pa)):
        job = W.workload_job(name)
        ts = []
        for k in range(3):
            t0 = time.perf_counter()
            gpu.submit_packed(job, L, lane=k & 1)
            ts.append(round((time.perf_counter() - t0) * 1e3, 3))
        out[name + "_ms"] = ts
    print(json.dumps(out), flush=True)
    gpu.close()


if __name__ == "__main__":
    main()
