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


def _chunk_worker(rank, world, port, out_path, n_pics):
    """bench.py --mode band's exchange on CPU: every rank searches its equal
    SB chunk of each of n_pics pictures, writes the records into its slice of
    a padded byte buffer and one all_gather_into_tensor per picture assembles
    every picture on every rank (RCCL moves device buffers the same way)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "svt-av1-mirror_amd"))
    import torch
    import torch.distributed as dist

    import svtme as S
    import svtme_dist as D

    dist.init_process_group("gloo", rank=rank, world_size=world)
    w, h = 200, 136  # 4 x 3 = 12 SBs: chunks of 6 at world 2 (5 + pad at world 3 would be short)
    n_sb = S.sb_total(w, h)
    R = 3
    # the split bench.py's band_8k leg uses (D.BandSplit: equal chunks, one all-gather)
    split = D.BandSplit(n_sb, R, S.REF_RECORD_DTYPE.itemsize, world, rank)
    outs = []
    for p in range(n_pics):
        ctrl = S.derive_controls(8, 35, S.input_resolution_of(w, h), 1)
        rec_bytes = S.REF_RECORD_DTYPE.itemsize * R
        local = torch.zeros(split.chunk_bytes, dtype=torch.uint8)
        if split.count:
            recs, _ = S.run_case_checker("pan", w, h, ctrl, 8 + p, (7 + p, 6 + p), (9 + p,), 1, checker="oracle",
                                         nthreads=1, sb_begin=split.begin, sb_count=split.count)
            local[: split.count * rec_bytes] = torch.from_numpy(recs.view(np.uint8).reshape(-1).copy())
        out = torch.empty(world * split.chunk_bytes, dtype=torch.uint8)
        split.exchange(local, out, dist)
        assert split.picture_bytes == n_sb * rec_bytes
        outs.append(split.picture(out).numpy().copy())
    if rank == 0:
        np.save(out_path, np.stack(outs))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_chunked_allgather_equals_single_rank(svtme, tmp_path, world):
    S = svtme
    out = str(tmp_path / "chunks.npy")
    mp.spawn(_chunk_worker, args=(world, _free_port(), out, 2), nprocs=world, join=True)
    got = np.load(out)
    w, h = 200, 136
    ctrl = S.derive_controls(8, 35, S.input_resolution_of(w, h), 1)
    for p in range(2):
        ref, _ = S.run_case_checker("pan", w, h, ctrl, 8 + p, (7 + p, 6 + p), (9 + p,), 1, checker="oracle",
                                    nthreads=2)
        full = got[p].view(S.REF_RECORD_DTYPE).reshape(ref.shape)
        assert not S.compare_records(ref, full)


def test_sb_chunk_padding():
    import svtme_dist as D

    for n in (1, 7, 12, 510, 2040, 8160):
        for world in (1, 2, 3, 4, 8):
            slots = D.chunk_slots(n, world)
            cov = []
            for k in range(world):
                b, c = D.sb_chunk(n, k, world)
                assert 0 <= c <= slots and b == min(k * slots, n)
                cov.extend(range(b, b + c))
            assert cov == list(range(n))


def _owner_worker(rank, world, port, out_path, k):
    """bench.py's default N > 1 exchange on CPU: world x k pictures per step,
    every rank searches its equal SB chunk of each, one all_to_all_single
    hands each picture's chunks to its owner rank (k pictures per rank)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "svt-av1-mirror_amd"))
    import torch
    import torch.distributed as dist

    import svtme as S
    import svtme_dist as D

    dist.init_process_group("gloo", rank=rank, world_size=world)
    w, h = 200, 136
    n_sb = S.sb_total(w, h)
    slots = D.chunk_slots(n_sb, world)
    R = 3
    rec_bytes = S.REF_RECORD_DTYPE.itemsize * R
    chunk = slots * rec_bytes
    n_pics = world * k
    ctrl = S.derive_controls(8, 35, S.input_resolution_of(w, h), 1)
    begin, count = D.sb_chunk(n_sb, rank, world)
    local = torch.zeros(n_pics * chunk, dtype=torch.uint8)
    for p in range(n_pics):
        if count:
            recs, _ = S.run_case_checker("pan", w, h, ctrl, 8 + p, (7 + p, 6 + p), (9 + p,), 1, checker="oracle",
                                         nthreads=1, sb_begin=begin, sb_count=count)
            local[p * chunk: p * chunk + count * rec_bytes] = torch.from_numpy(recs.view(np.uint8).reshape(-1).copy())
    out = torch.empty_like(local)
    D.exchange_to_owners_device(local, out, dist)
    for q in range(k):
        p = rank * k + q
        assert D.owner_of(p, k) == rank
        got = D.owned_picture_records(out, world, k, q, n_sb * rec_bytes)
        np.save(f"{out_path}.{p}.npy", got.numpy().copy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,k", [(2, 2), (3, 1)])
def test_owner_exchange_equals_single_rank(svtme, tmp_path, world, k):
    S = svtme
    out = str(tmp_path / "owned")
    mp.spawn(_owner_worker, args=(world, _free_port(), out, k), nprocs=world, join=True)
    w, h = 200, 136
    ctrl = S.derive_controls(8, 35, S.input_resolution_of(w, h), 1)
    for p in range(world * k):
        ref, _ = S.run_case_checker("pan", w, h, ctrl, 8 + p, (7 + p, 6 + p), (9 + p,), 1, checker="oracle",
                                    nthreads=2)
        full = np.load(f"{out}.{p}.npy").view(S.REF_RECORD_DTYPE).reshape(ref.shape)
        assert not S.compare_records(ref, full)


def _bcast_worker(rank, world, port, out_path, n_pics, mode="broadcast"):
    """bench.py's band_8k step on CPU: rank 0 holds the current picture's luma
    plane, one broadcast (svtme_dist.broadcast_plane) gives it to every rank,
    every rank builds the pyramid from what it received, searches its equal SB
    chunk against its resident references and one all_gather_into_tensor
    assembles the picture's records on every rank."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "svt-av1-mirror_amd"))
    import torch
    import torch.distributed as dist

    import svtme as S
    import svtme_dist as D

    dist.init_process_group("gloo", rank=rank, world_size=world)
    w, h = 264, 200  # 5 x 4 = 20 SBs, ragged width and height
    n_sb = S.sb_total(w, h)
    R = 3
    split = D.BandSplit(n_sb, R, S.REF_RECORD_DTYPE.itemsize, world, rank)
    ctrl = S.derive_controls(8, 35, S.input_resolution_of(w, h), 1)
    outs = []
    for p in range(n_pics):
        cur = 8 + 3 * p
        frames = S.test_frames("pan", w, h, [cur - 1, cur - 2, cur, cur + 1])
        refs = {(0, 0): S.build_host_pyramid(frames[cur - 1]), (0, 1): S.build_host_pyramid(frames[cur - 2]),
                (1, 0): S.build_host_pyramid(frames[cur + 1])}  # resident: distributed with earlier pictures
        if mode == "broadcast":
            plane = torch.from_numpy(frames[cur].copy()) if rank == 0 else torch.zeros((h, w), dtype=torch.uint8)
            D.broadcast_plane(plane, dist, src=0)
        else:  # sliced: each rank holds (uploads) only its rows; one all-gather assembles the plane
            ps = D.PlaneSlices(w, h, world, rank)
            sl = torch.zeros(ps.slice_bytes, dtype=torch.uint8)
            mine = torch.from_numpy(ps.host_rows(frames[cur]).copy())
            sl[: mine.numel()] = mine
            full = torch.zeros(ps.plane_bytes, dtype=torch.uint8)
            ps.gather(sl, full, dist)
            plane = full[: h * w].reshape(h, w)
        local = torch.zeros(split.chunk_bytes, dtype=torch.uint8)
        if split.count:
            job = S.case_job(ctrl, w, h, cur, (cur - 1, cur - 2), (cur + 1,), 1, sb_begin=split.begin,
                             sb_count=split.count)
            recs, _ = S.run_checker(job, S.build_host_pyramid(plane.numpy()), refs, "oracle", nthreads=1,
                                    with_sb_results=False)
            local[: recs.nbytes] = torch.from_numpy(recs.view(np.uint8).reshape(-1).copy())
        out = torch.empty(world * split.chunk_bytes, dtype=torch.uint8)
        split.exchange(local, out, dist)
        outs.append(split.picture(out).numpy().copy())
    np.save(f"{out_path}.{rank}.npy", np.stack(outs))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["broadcast", "sliced"])
@pytest.mark.parametrize("world", [2, 3])
def test_broadcast_chunked_search_allgather_equals_single_rank(svtme, tmp_path, world, mode):
    """The input either broadcast from rank 0 or uploaded in row slices (each
    rank its own rows, svtme_dist.PlaneSlices) and all-gathered; then the
    chunked search and the record all-gather: bit-identical to one rank."""
    S = svtme
    out = str(tmp_path / "bcast")
    mp.spawn(_bcast_worker, args=(world, _free_port(), out, 2, mode), nprocs=world, join=True)
    w, h = 264, 200
    ctrl = S.derive_controls(8, 35, S.input_resolution_of(w, h), 1)
    for rank in range(world):  # every rank holds every picture's records
        got = np.load(f"{out}.{rank}.npy")
        for p in range(2):
            cur = 8 + 3 * p
            ref, _ = S.run_case_checker("pan", w, h, ctrl, cur, (cur - 1, cur - 2), (cur + 1,), 1, checker="oracle",
                                        nthreads=2)
            full = got[p].view(S.REF_RECORD_DTYPE).reshape(ref.shape)
            assert not S.compare_records(ref, full)
