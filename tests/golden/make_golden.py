"""Generate the golden fixtures under tests/golden/ from the reference itself.

The reference's own open-loop ME (motion_estimation.c and the kernels it
dispatches to) and its svt_aom_sig_deriv_me (enc_mode_config.c) are compiled
from the sources under /root/reference into oracle/_ref/libsvtref.so by
oracle/Makefile (`make -C oracle ref`). This script drives that library on
deterministic inputs (svtme.test_frames / the PCG32 synthetic texture) and
stores inputs-as-parameters plus expected outputs:

  controls.json      svt_aom_sig_deriv_me outputs over presets x resolutions x
                     temporal layers x QPs (the product restates it in C++)
  me_cases.json      the ME cases (content, size, preset, layer, references)
  me_<name>.npz      expected per-SB reference records and SB results
                     (raw bytes of REF_RECORD_DTYPE / SB_RESULT_DTYPE), plus
                     sha256 digests of the reference's padded pyramids
  controls_tf.json   svt_aom_sig_deriv_me_tf outputs (TF-ME controls) over
                     hme_me_level x qp_opt x QP x resolution
  tf_cases.json      temporal-filtering ME cases (me_type ME_MCTF: one list,
                     one reference, HME-only exits) -> me_tf_<name>.npz
  configs.json       the BASELINE.json configurations at full size
                     (svt-av1-mirror_amd/workloads.py): record/SB-result checksums
                     of the whole picture plus every STRIDE-th SB's records in
                     cfg_<name>.npz; configs[0] (640x360 p12, 30 pictures random
                     access) as per-picture checksums and full records

Run from the repo root in the build container (needs /root/reference for the
library build only): python tests/golden/make_golden.py [tf|me|configs [name ...]|rtcd]
(tf / me / configs / rtcd: only those fixtures; configs name ...: only those configurations)
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "svt-av1-mirror_amd"))

import svtme as S  # noqa: E402

ME_CASES = [
    # name, content, w, h, preset, tl, l0, l1, extra
    ("pan320_p8_tl1", "pan", 320, 192, 8, 1, (7, 6), (9, 10), {}),
    ("pan640_p4_tl2", "pan", 640, 360, 4, 2, (7, 6), (9,), {}),
    ("pan426_p6_tl0", "pan", 426, 240, 6, 0, (7, 6, 5), (9, 10), {}),
    ("pan72_p8_edges", "pan", 72, 40, 8, 1, (7, 6), (9, 10), {}),
    ("pan136x8_p6", "pan", 136, 8, 6, 1, (7,), (9,), {}),
    ("noise320_p12_single", "noise", 320, 192, 12, 0, (7,), (), {}),
    ("flat320_p4_ties", "flat", 320, 192, 4, 1, (7,), (9,), {}),
    ("sat192_p6", "sat", 192, 128, 6, 1, (7, 6), (9,), {}),
    ("stripes320_p8_7refs", "stripes", 320, 192, 8, 3, (7, 6, 4, 3), (9, 10, 12), {}),
    ("pan640_p4_gm", "pan", 640, 360, 4, 1, (7, 6), (9,), {"gm": True}),
    ("pan320_p8_band", "pan", 320, 192, 8, 1, (7, 6), (9, 10), {"sb_begin": 3, "sb_count": 7}),
    ("pan64_p0", "pan", 64, 64, 0, 1, (7,), (9,), {}),
    ("pan320_p8_nonref", "pan", 320, 192, 8, 2, (7,), (9,), {"is_ref": False}),
    # real-time tune (low-delay prediction, enc_mode_config.c:692-704): HME-L0 areas
    # of every slot but the first follow the first slot's HME-L0 centre
    # (motion_estimation.c:1800-1867); "ctrl" overrides fields of the derived controls
    ("pan320_p8_rt200", "pan", 320, 192, 8, 1, (7, 6), (9, 10),
     {"ctrl": {"reduce_hme_l0_sr_th_min": 8, "reduce_hme_l0_sr_th_max": 200}}),
    ("vpan640_p8_rt100", "vpan", 640, 360, 8, 1, (7, 6, 5), (9,),
     {"ctrl": {"reduce_hme_l0_sr_th_min": 8, "reduce_hme_l0_sr_th_max": 100}}),
    ("hpan640_p9_rt100", "hpan", 640, 360, 9, 2, (7, 6), (9, 10),
     {"ctrl": {"reduce_hme_l0_sr_th_min": 8, "reduce_hme_l0_sr_th_max": 100}}),
    ("vpan640_p8_rt100_adj2", "vpan", 640, 360, 8, 1, (7, 6), (9, 10),
     {"ctrl": {"reduce_hme_l0_sr_th_min": 8, "reduce_hme_l0_sr_th_max": 100, "enable_me_sr_adjustment": 2}}),
    ("pan640_p8_rt200_adj2", "pan", 640, 360, 8, 1, (7, 6, 5), (9, 10),
     {"ctrl": {"reduce_hme_l0_sr_th_min": 8, "reduce_hme_l0_sr_th_max": 200, "enable_me_sr_adjustment": 2}}),
    # a width that is not a multiple of 64: the split HME path's two stage-A rounds
    ("vpan424_p8_rt100", "vpan", 424, 240, 8, 1, (7, 6), (9, 10),
     {"ctrl": {"reduce_hme_l0_sr_th_min": 8, "reduce_hme_l0_sr_th_max": 100}}),
]

TF_CASES = [
    # name, content, w, h, tf hme_me_level, qp_opt, qp, cur, ref, tl, tf_me_exit_th
    ("tf_pan320_lvl0", "pan", 320, 192, 0, 0, 35, 8, 7, 1, 0),
    ("tf_pan320_lvl1_fwd2", "pan", 320, 192, 1, 0, 35, 8, 10, 1, 0),
    ("tf_pan640_lvl2_qp20_exit", "pan", 640, 360, 2, 1, 20, 8, 9, 0, 9800),
    ("tf_pan320_lvl3_exit", "pan", 320, 192, 3, 0, 35, 8, 7, 1, 2600),
    ("tf_noise192_lvl3", "noise", 192, 128, 3, 0, 35, 8, 6, 2, 0),
    ("tf_flat192_lvl4_exit", "flat", 192, 128, 4, 0, 35, 8, 7, 1, 1),
    ("tf_stripes320_lvl2_exit", "stripes", 320, 192, 2, 0, 35, 8, 9, 1, 50000),
]

CTRL_GRID = dict(enc_mode=list(range(14)), input_resolution=list(range(7)), tl=[0, 1, 2, 3], qp=[35, 55])


def controls_golden():
    unique, index, rows = [], {}, []
    for m in CTRL_GRID["enc_mode"]:
        for res in CTRL_GRID["input_resolution"]:
            for tl in CTRL_GRID["tl"]:
                for qp in CTRL_GRID["qp"]:
                    d = S.ref_derive_controls(m, qp, res, tl).as_dict()
                    key = json.dumps(d, sort_keys=True)
                    if key not in index:
                        index[key] = len(unique)
                        unique.append(d)
                    rows.append([m, qp, res, tl, index[key]])
    return {"args": ["enc_mode", "qp", "input_resolution", "temporal_layer_index", "unique_index"],
            "unique": unique, "rows": rows}


def digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def rtcd_golden():
    """Per-kernel outputs of the reference's C kernels (AVX2 must agree)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import rtcd_cases as R

    ref = S.load_ref()
    out = {}
    for name, run in R.all_cases():
        ref.svtref_set_simd(0)
        a = run(ref, "svtref_")
        ref.svtref_set_simd(1)
        b = run(ref, "svtref_")
        for k in a:
            assert np.array_equal(a[k], b[k]), (name, k)
            out[f"{name}/{k}"] = a[k]
    np.savez_compressed(os.path.join(HERE, "rtcd_cases.npz"), **out)
    print("rtcd cases", len(out))


def tf_golden():
    """TF-ME (me_type ME_MCTF) fixtures: controls of svt_aom_sig_deriv_me_tf and
    the reference's svt_aom_motion_estimation_b64 run as temporal_filtering.c:3127-3174
    runs it (one list, one reference)."""
    ref = S.load_ref()
    unique, index, rows = [], {}, []
    for lvl in range(5):
        for qp_opt in (0, 1):
            for qp in (10, 20, 35, 55):
                for res in range(7):
                    d = S.ref_derive_controls_tf(lvl, qp_opt, qp, res).as_dict()
                    key = json.dumps(d, sort_keys=True)
                    if key not in index:
                        index[key] = len(unique)
                        unique.append(d)
                    rows.append([lvl, qp_opt, qp, res, index[key]])
    with open(os.path.join(HERE, "controls_tf.json"), "w") as fh:
        json.dump({"args": ["hme_me_level", "qp_opt", "qp", "input_resolution", "unique_index"], "unique": unique,
                   "rows": rows}, fh, indent=0)
    meta = []
    for name, kind, w, h, lvl, qp_opt, qp, cur, refp, tl, th in TF_CASES:
        ctrl = S.ref_derive_controls_tf(lvl, qp_opt, qp, S.input_resolution_of(w, h))
        extra = {"me_type": S.ME_MCTF, "tf_me_exit_th": th}
        out = {}
        for simd in (0, 1):  # C kernels and AVX2 kernels must agree
            ref.svtref_set_simd(simd)
            out[simd] = S.run_case_checker(kind, w, h, ctrl, cur, (refp,), (), tl, checker="ref", **extra)
        recs, sbr = out[0]
        assert not S.compare_records(recs, out[1][0], sbr, out[1][1]), name
        np.savez_compressed(os.path.join(HERE, f"me_{name}.npz"), records=recs.view(np.uint8).reshape(len(recs), -1),
                            sb=sbr.view(np.uint8).reshape(len(sbr), -1))
        meta.append({"name": name, "content": kind, "w": w, "h": h, "cur": cur, "tl": tl, "l0": [refp], "l1": [],
                     "hme_me_level": lvl, "qp_opt": qp_opt, "qp": qp, "ctrl": ctrl.as_dict(), "extra": extra,
                     "checksum": S.records_checksum(recs, sbr), "tf_exits": int(recs["tf_early_exit"].sum())})
        print(name, recs.shape, "exits", meta[-1]["tf_exits"], meta[-1]["checksum"][:16])
    with open(os.path.join(HERE, "tf_cases.json"), "w") as fh:
        json.dump(meta, fh, indent=1)


CFG_STRIDE = 7  # sampled SBs of the full-size configurations (every 7th SB: all rows and columns)


CFG_NAMES = ("1080p_sa64", "4k_p8", "4k10_p6", "8k_p8", "4k_p8_mixed")


def configs_golden(only=None):
    """Full-size BASELINE.json configurations through the reference's own ME
    (AVX2 kernels, as the encoder runs at --asm avx2; the C kernels must agree
    on the sampled SBs of every configuration). only: regenerate just these
    configurations and keep the others' entries of configs.json."""
    import workloads as W

    ref = S.load_ref()
    meta = {"stride": CFG_STRIDE, "configs": {}, "ra360_p12": []}
    if only:
        with open(os.path.join(HERE, "configs.json")) as fh:
            meta = json.load(fh)
    for name in (only or CFG_NAMES):
        wl = W.WORKLOADS[name]
        frames = W.workload_frames(name)
        pyr = {t: S.build_host_pyramid(f, "ref") for t, f in frames.items()}
        refs = {(0, i): pyr[t] for i, t in enumerate(wl["l0"])}
        refs.update({(1, i): pyr[t] for i, t in enumerate(wl["l1"])})
        job = W.workload_job(name)
        ref.svtref_set_simd(1)
        recs, sbr = S.run_checker(job, pyr[8], refs, "ref", nthreads=8)
        # C kernels on the sampled SBs (one band job per sample keeps the C run short)
        ref.svtref_set_simd(0)
        n = len(recs)
        for b in range(0, n, CFG_STRIDE * 16):
            cj = W.workload_job(name, sb_begin=b, sb_count=1)
            crec, csb = S.run_checker(cj, pyr[8], refs, "ref", nthreads=1)
            assert not S.compare_records(recs[b:b + 1], crec, sbr[b:b + 1], csb), (name, b)
        ref.svtref_set_simd(1)
        np.savez_compressed(os.path.join(HERE, f"cfg_{name}.npz"),
                            records=np.ascontiguousarray(recs[::CFG_STRIDE]).view(np.uint8).reshape(-1, recs.shape[1] * recs.itemsize),
                            sb=np.ascontiguousarray(sbr[::CFG_STRIDE]).view(np.uint8).reshape(-1, sbr.itemsize))
        meta["configs"][name] = {"sbs": n, "refs": int(recs.shape[1]), "checksum": S.records_checksum(recs, sbr),
                                 "searched": int(recs["searched"].sum()), "desc": wl["desc"],
                                 "pyramid_sha256": digest(pyr[8].full)}
        print(name, recs.shape, meta["configs"][name]["checksum"][:16], flush=True)
    if only:
        with open(os.path.join(HERE, "configs.json"), "w") as fh:
            json.dump(meta, fh, indent=1)
        return
    # configs[0]: 640x360 preset 12, 30 pictures random access
    w, h = 640, 360
    syn = S.Synth(w, h)
    frames = {t: syn.frame(t) for t in range(30)}
    pyr = {t: S.build_host_pyramid(f, "ref") for t, f in frames.items()}
    all_recs, all_sb = [], []
    for t, tl, l0, l1 in W.ra_sequence(30):
        ctrl = S.ref_derive_controls(12, 35, S.input_resolution_of(w, h), tl)
        job = S.case_job(ctrl, w, h, t, l0, l1, tl)
        refs = {(0, i): pyr[u] for i, u in enumerate(l0)}
        refs.update({(1, i): pyr[u] for i, u in enumerate(l1)})
        recs, sbr = S.run_checker(job, pyr[t], refs, "ref", nthreads=8)
        meta["ra360_p12"].append({"picture": t, "tl": tl, "l0": list(l0), "l1": list(l1),
                                  "checksum": S.records_checksum(recs, sbr)})
        all_recs.append(recs.view(np.uint8).reshape(-1))
        all_sb.append(sbr.view(np.uint8).reshape(-1))
    np.savez_compressed(os.path.join(HERE, "cfg_ra360_p12.npz"), records=np.concatenate(all_recs),
                        sb=np.concatenate(all_sb))
    with open(os.path.join(HERE, "configs.json"), "w") as fh:
        json.dump(meta, fh, indent=1)


def case_controls(preset, w, h, tl, extra):
    """svt_aom_sig_deriv_me's controls of a case, with the case's overrides"""
    ctrl = S.ref_derive_controls(preset, 35, S.input_resolution_of(w, h), tl)
    for k, v in extra.get("ctrl", {}).items():
        setattr(ctrl, k, v)
    return ctrl


def main():
    ref = S.load_ref()
    rtcd_golden()
    with open(os.path.join(HERE, "controls.json"), "w") as fh:
        json.dump(controls_golden(), fh, indent=0)
    me_golden(ref)


def me_golden(ref):
    meta = []
    for name, kind, w, h, preset, tl, l0, l1, extra in ME_CASES:
        ctrl = case_controls(preset, w, h, tl, extra)
        extra = {k: v for k, v in extra.items() if k != "ctrl"}
        out = {}
        for simd in (0, 1):  # C kernels and AVX2 kernels must agree
            ref.svtref_set_simd(simd)
            out[simd] = S.run_case_checker(kind, w, h, ctrl, 8, l0, l1, tl, checker="ref", **extra)
        recs, sbr = out[0]
        assert not S.compare_records(recs, out[1][0], sbr, out[1][1]), name
        frames = S.test_frames(kind, w, h, [8])
        p = S.build_host_pyramid(frames[8], "ref")
        np.savez_compressed(os.path.join(HERE, f"me_{name}.npz"), records=recs.view(np.uint8).reshape(len(recs), -1),
                            sb=sbr.view(np.uint8).reshape(len(sbr), -1))
        meta.append({"name": name, "content": kind, "w": w, "h": h, "preset": preset, "tl": tl, "l0": list(l0), "ctrl": ctrl.as_dict(),
                     "l1": list(l1), "extra": extra, "checksum": S.records_checksum(recs, sbr),
                     "pyramid_sha256": {k: digest(getattr(p, k)) for k in ("full", "quarter", "sixteenth")}})
        print(name, recs.shape, meta[-1]["checksum"][:16])
    with open(os.path.join(HERE, "me_cases.json"), "w") as fh:
        json.dump(meta, fh, indent=1)


if __name__ == "__main__":
    if sys.argv[1:] == ["configs"]:
        configs_golden()
    elif sys.argv[1:2] == ["configs"]:
        configs_golden(sys.argv[2:])
    elif sys.argv[1:] == ["rtcd"]:
        rtcd_golden()
    elif sys.argv[1:] == ["me"]:
        me_golden(S.load_ref())
    else:
        if sys.argv[1:] != ["tf"]:
            main()
        tf_golden()
        configs_golden()
