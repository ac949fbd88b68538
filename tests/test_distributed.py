"""CPU multi-process coverage of the N > 1 path (gloo, world_size 2, 127.0.0.1).

Band-parallel ME of one picture: each rank searches its SB band with the
checker backend, the bands are all-gathered (svtme_dist.gather_band_records)
and must equal the single-rank picture bit-exactly. The GPU build runs the
same orchestration with libsvtme.so and RCCL; bench.py's picture-parallel
mode needs no exchange at all.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "svt-av1-mirror_amd"))
    import torch.distributed as dist

    import svtme as S
    import svtme_dist as D

    dist.init_process_group("gloo", rank=rank, world_size=world)
    w, h = 320, 192
    ctrl = S.derive_controls(8, 35, S.input_resolution_of(w, h), 1)
    n_sb = S.sb_total(w, h)
    begin, count = D.sb_band(n_sb, rank, world)
    recs, _ = S.run_case_checker("pan", w, h, ctrl, 8, (7, 6), (9, 10), 1, checker="oracle", nthreads=2,
                                 sb_begin=begin, sb_count=count)
    full = D.gather_band_records(recs, n_sb, dist)
    if rank == 0:
        np.save(out_path, full.view(np.uint8))
    dist.barrier()
    dist.destroy_process_group()


def test_sb_band_partition():
    import svtme_dist as D

    for n in (1, 7, 15, 2040):
        for world in (1, 2, 3, 8):
            bands = [D.sb_band(n, k, world) for k in range(world)]
            assert bands[0][0] == 0 and sum(c for _, c in bands) == n
            for (b0, c0), (b1, _) in zip(bands, bands[1:]):
                assert b0 + c0 == b1


def test_band_parallel_equals_single_rank(svtme, tmp_path):
    S = svtme
    out = str(tmp_path / "full.npy")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    full = np.load(out).view(S.REF_RECORD_DTYPE).reshape(S.sb_total(320, 192), -1)
    ctrl = S.derive_controls(8, 35, S.input_resolution_of(320, 192), 1)
    ref, _ = S.run_case_checker("pan", 320, 192, ctrl, 8, (7, 6), (9, 10), 1, checker="oracle", nthreads=2)
    assert not S.compare_records(ref, full)
