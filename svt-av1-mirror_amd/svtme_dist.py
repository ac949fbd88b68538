"""Multi-GPU orchestration of the open-loop ME path (one process per GPU).

Two ways to spread ME over ranks, neither needs a collective on the data path:

* picture-parallel (weak scaling, what bench.py measures): every rank runs
  whole pictures of its own; the only exchange is the optional all-gather of
  the per-SB records (the encoder's picture-level consumers, me_process.c:
  274-288, read every SB's results).
* band-parallel (one picture split in SB-row bands): rank k runs SBs
  [begin_k, begin_k + count_k) of the same picture (svtme_job.sb_begin /
  sb_count) against the same resident references; the bands concatenate to
  the whole picture's records, bit-identical to a single-rank run.

`torch.distributed` is plumbing here (RCCL on GPUs, gloo for the CPU tests).
"""
import numpy as np


def sb_band(n_sb: int, rank: int, world: int):
    """Contiguous SB band of `rank`: whole SB rows are not required, only
    contiguity (records are indexed by picture-raster SB number)."""
    q, r = divmod(n_sb, world)
    begin = rank * q + min(rank, r)
    return begin, q + (1 if rank < r else 0)


def gather_band_records(local: np.ndarray, n_sb: int, dist, group=None) -> np.ndarray:
    """All-gather the per-rank record bands (structured numpy arrays of shape
    [count_k, R]) into the picture's [n_sb, R] array on every rank."""
    import torch

    world = dist.get_world_size(group)
    R = local.shape[1]
    itemsize = local.dtype.itemsize
    counts = [sb_band(n_sb, k, world)[1] for k in range(world)]
    maxc = max(counts)
    buf = np.zeros((maxc, R), local.dtype)
    buf[: local.shape[0]] = local
    t = torch.from_numpy(buf.view(np.uint8).reshape(-1).copy())
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t, group=group)
    parts = [o.numpy().view(local.dtype).reshape(maxc, R)[:c] for o, c in zip(out, counts)]
    res = np.concatenate(parts, axis=0)
    assert res.shape[0] == n_sb and res.dtype.itemsize == itemsize
    return res
