# Low-delay (real-time tune) preset sweep of the glue over the oracle-backed job API: every
# preset 7-13 at 640x360 and 426x240, bitstreams compared with the unmodified encoder (CPU).
import sys, json
sys.path.insert(0, "tests")
import encoder_harness as E
res = []
for w, h, tag in ((640, 360, "360"), (426, 240, "240")):
    for p in range(7, 14):
        name = f"ld{tag}_p{p}"
        E.CASES[name] = (w, h, 12, p, False, ["--pred-struct", "1"], True)
        r = E.check(name, "ora", "/tmp/svtme_enc")
        res.append((name, r["md5"][:8], r["sbs"], r["fallback_sbs"]))
        print(res[-1], flush=True)
