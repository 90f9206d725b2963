"""Row-interleaved partition of one image over ranks + the final gather to rank 0.

SURVEY §8(e): pixels are independent, so rendering needs no exchange; row j goes to rank
j mod world (interleaving spreads cheap sky rows and expensive ground rows evenly).  The one
collective is the final gather of every rank's rows to rank 0 (RCCL over xGMI with the "nccl"
backend on ROCm; gloo on CPU in tests).  The RNG is keyed by the global pixel index, so the
gathered image is bit-identical for any world size.
"""
import torch
import torch.distributed as dist


def rows_per_rank(height, world):
    """Padded per-rank row count R = ceil(H / world); rank r owns rows r, r+world, ..."""
    return (height + world - 1) // world


def rank_rows(height, rank, world):
    """(row0, row_step, n_rows) for this rank's interleaved rows."""
    n = (height - rank + world - 1) // world if rank < height else 0
    return rank, world, n


def assemble(gathered, height):
    """gathered: (world, R, W, C) with slot [r][k] = row r + k*world -> (H, W, C) image."""
    world, R = gathered.shape[0], gathered.shape[1]
    img = gathered.transpose(0, 1).reshape(R * world, *gathered.shape[2:])
    return img[:height]


def gather_image(local, height, rank, world, group=None, collective=False):
    """local: (R, W, C) padded rows of this rank (rows beyond its n_rows are ignored).
    Returns the (H, W, C) image on rank 0 and None elsewhere.  At world 1 the rows are the image;
    collective=True still runs the gather through the process group (bench.py --collective: the
    RCCL path exercised on a 1-GPU box with a 1-rank nccl group)."""
    if world == 1 and not collective:
        return local[:height]
    if rank == 0:
        # the peers' rows land in views of ONE (world, R, W, C) buffer: no stack copy
        buf = torch.empty((world,) + tuple(local.shape), dtype=local.dtype, device=local.device)
        dist.gather(local, gather_list=list(buf.unbind(0)), dst=0, group=group)
        return assemble(buf, height)
    dist.gather(local, dst=0, group=group)
    return None
