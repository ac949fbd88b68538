"""Multi-GPU orchestration of the open-loop ME path (one process per GPU).

Two ways to spread ME over ranks:

* picture-parallel: every rank runs whole pictures of its own; no exchange.
* band-parallel (one picture split in SB bands): rank k runs
  SBs [begin_k, begin_k + count_k) of the same picture (svtme_job.sb_begin /
  sb_count) against the same resident references; the bands concatenate to
  the whole picture's records, bit-identical to a single-rank run. On GPUs the
  SB count is padded to equal chunks (sb_chunk) so one all_gather_into_tensor
  over RCCL moves every rank's record slice straight between device buffers
  (gather_chunks_device), or, with several pictures per step, one
  all_to_all_single hands each picture's chunks to the rank that owns it
  (exchange_to_owners_device); this is the analogue of the reference's ME segments
  -> SB ranges (enc_handle.c:393-412, me_process.c:146-157).

`torch.distributed` is plumbing here (RCCL on GPUs, gloo for the CPU tests).
"""
import numpy as np


def sb_band(n_sb: int, rank: int, world: int):
    """Contiguous SB band of `rank`: whole SB rows are not required, only
    contiguity (records are indexed by picture-raster SB number)."""
    q, r = divmod(n_sb, world)
    begin = rank * q + min(rank, r)
    return begin, q + (1 if rank < r else 0)


def sb_chunk(n_sb: int, rank: int, world: int):
    """Equal-chunk band of `rank`: chunk = ceil(n_sb / world) SBs, the last
    rank(s) short (count may be 0). Every rank's slice of the gathered buffer
    has the same size, so the exchange is a single all-gather."""
    chunk = -(-n_sb // world)
    begin = min(rank * chunk, n_sb)
    return begin, max(0, min(chunk, n_sb - begin))


def chunk_slots(n_sb: int, world: int) -> int:
    """SB slots per rank in the padded all-gather buffer."""
    return -(-n_sb // world)


class BandSplit:
    """One picture's SBs over the ranks: rank r searches the
    equal chunk r (sb_chunk) into a local buffer of `chunk_bytes`; one
    all_gather_into_tensor assembles the picture's records, in raster SB
    order, in the first `picture_bytes` of every rank's gathered buffer."""

    def __init__(self, n_sb: int, refs: int, record_bytes: int, world: int, rank: int):
        self.n_sb, self.world, self.rank = n_sb, world, rank
        self.slots = chunk_slots(n_sb, world)
        self.begin, self.count = sb_chunk(n_sb, rank, world)
        self.chunk_bytes = self.slots * refs * record_bytes
        self.picture_bytes = n_sb * refs * record_bytes
        # bytes each rank receives per picture (its own chunk is already local)
        self.gather_bytes_in = (world - 1) * self.chunk_bytes

    def exchange(self, d_local, d_out, dist, stream=None):
        if self.world == 1:
            return d_local
        return gather_chunks_device(d_local, d_out, dist, stream=stream)

    def picture(self, d_out):
        return d_out[: self.picture_bytes]


def broadcast_plane(plane, dist, src: int = 0, group=None, stream=None):
    """SURVEY.md 8(e) input distribution: the current picture's 8-bit luma plane
    (uint8 tensor) from rank `src` to every rank of the split, one broadcast
    (RCCL over xGMI on GPUs, on `stream`; gloo in the CPU tests). Every rank
    then builds the picture's pyramid from it (svtme_picture_upload_device_async)."""
    import torch

    if stream is not None:
        with torch.cuda.stream(stream):
            dist.broadcast(plane, src=src, group=group)
    else:
        dist.broadcast(plane, src=src, group=group)
    return plane


class PlaneSlices:
    """SURVEY.md 8(e) input distribution that scales with the ranks: rank r
    copies rows [r * rows, (r + 1) * rows) of the current H x W luma plane
    (rows = ceil(H / world)) from host memory over ITS OWN PCIe link into a
    device slice, and one all_gather_into_tensor over xGMI assembles the whole
    plane on every rank (the gathered buffer holds world x rows rows; those past
    H are padding nobody reads). Each rank then builds the pyramid from it
    (svtme_picture_upload_device_async). PCIe bytes per rank: H W / world,
    against H W for every rank uploading the whole plane or for rank 0 before a
    broadcast."""

    def __init__(self, width: int, height: int, world: int, rank: int):
        self.w, self.h, self.world, self.rank = width, height, world, rank
        self.rows = -(-height // world)
        self.r0 = min(rank * self.rows, height)
        self.r1 = min(height, self.r0 + self.rows)
        self.slice_bytes = self.rows * width
        self.plane_bytes = world * self.slice_bytes

    def host_rows(self, frame):
        """This rank's rows of the plane (a view of the H x W frame, flattened)."""
        return frame[self.r0: self.r1].reshape(-1)

    def gather(self, d_slice, d_plane, dist, group=None, stream=None):
        """d_slice: uint8 tensor of slice_bytes (this rank's rows first);
        d_plane: uint8 tensor of plane_bytes; its first H x W bytes are the plane."""
        if self.world == 1:
            d_plane[: self.slice_bytes].copy_(d_slice)
            return d_plane
        return gather_chunks_device(d_slice, d_plane, dist, group=group, stream=stream)


def gather_chunks_device(d_local, d_out, dist, group=None, stream=None):
    """All-gather the ranks' record chunks between device buffers.

    d_local: uint8 tensor of chunk_slots x R x record bytes (this rank's
    records, written by svtme_submit_picture_device; a short last chunk leaves
    its tail unused); d_out: uint8 tensor world x that size. Row-major SB
    order of the picture is d_out[:n_sb * R * record bytes]. With RCCL
    the copy runs on `stream` (the ME library's stream, so it is ordered after
    the ME kernels without a host sync)."""
    import torch

    if stream is not None:
        with torch.cuda.stream(stream):
            dist.all_gather_into_tensor(d_out, d_local, group=group)
    else:
        dist.all_gather_into_tensor(d_out, d_local, group=group)
    return d_out


def owner_of(picture: int, pictures_per_rank: int) -> int:
    """Rank that assembles `picture` (of a step's world x pictures_per_rank
    pictures, numbered so that each rank's pictures are contiguous)."""
    return picture // pictures_per_rank


def exchange_to_owners_device(d_local, d_out, dist, group=None, stream=None):
    """Send each picture's record chunk to the rank that owns the picture.

    A step has world x k pictures; rank j owns pictures [j k, (j + 1) k) (the
    encoder process whose picture-level consumers read every SB's records of
    that picture, me_process.c:274-288). d_local: uint8 tensor of world x k
    chunks (this rank's chunk of every picture, picture-major); d_out: the same
    size, chunk i of owned picture q at d_out[(i k + q) chunk : ...]
    (owned_picture_records reassembles it). One all_to_all_single over RCCL:
    each rank moves (world - 1) / world of k pictures' records instead of the
    (world - 1) x world x k chunks an all-gather moves to every rank."""
    import torch

    if stream is not None:
        with torch.cuda.stream(stream):
            dist.all_to_all_single(d_out, d_local, group=group)
    else:
        dist.all_to_all_single(d_out, d_local, group=group)
    return d_out


def owned_picture_records(d_out, world: int, pictures_per_rank: int, q: int, n_bytes: int):
    """The records (first n_bytes: n_sb x R x record bytes, raster SB order) of
    this rank's q-th owned picture out of exchange_to_owners_device's buffer."""
    chunk = d_out.numel() // (world * pictures_per_rank)
    return d_out.view(world, pictures_per_rank, chunk)[:, q, :].reshape(-1)[:n_bytes]


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
    if dist.get_backend(group) == "nccl":  # RCCL moves device tensors only
        t = t.cuda()
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t, group=group)
    parts = [o.cpu().numpy().view(local.dtype).reshape(maxc, R)[:c] for o, c in zip(out, counts)]
    res = np.concatenate(parts, axis=0)
    assert res.shape[0] == n_sb and res.dtype.itemsize == itemsize
    return res
