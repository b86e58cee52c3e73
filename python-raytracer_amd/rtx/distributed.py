"""Multi-GPU frame rendering: one process per GPU, row blocks, one gather.

The reference parallelises by rendering column strips in separate processes and
stitching them on the filesystem (render.nu:2-23, provided/main.py:26-28,
provided/glue.py:17-27). Here each rank renders the row block
``np.array_split(np.arange(H), world)[rank]`` of the final image on its own GPU (the
camera tables are global, so results do not depend on the partition) and the blocks are
gathered to rank 0 with one collective (RCCL over xGMI on MI355X; gloo in CPU tests).
Blocks are padded to ceil(H / world) rows so the gather moves equal-sized buffers.
With ``interleave=True`` each rank instead renders the 8-row groups rank, rank + world, ...
(``rtx_render_groups``), which balances the sky/ground cost across ranks; rank 0 scatters
the gathered groups back into place.
"""
import torch
import torch.distributed as dist

from .scene import group_rows, split_rows


def row_block(height, world, rank):
    return split_rows(height, world, rank)


def gather_rows(block, height, world, rank, dst=0, group=None):
    """Gather per-rank row blocks [nrows_r, W, C] into the full [height, W, C] frame on
    ``dst`` (returns None on other ranks). Works for any dtype/device the backend takes."""
    maxrows = -(-height // world)
    _, nrows = split_rows(height, world, rank)
    if block.shape[0] != nrows:
        raise ValueError("rank %d block has %d rows, expected %d" % (rank, block.shape[0], nrows))
    if nrows == maxrows:
        send = block.contiguous()
    else:
        send = torch.zeros((maxrows,) + tuple(block.shape[1:]), dtype=block.dtype, device=block.device)
        send[:nrows] = block
    if rank == dst:
        bufs = [torch.empty_like(send) for _ in range(world)]
        dist.gather(send, gather_list=bufs, dst=dst, group=group)
        parts = []
        for r in range(world):
            _, nr = split_rows(height, world, r)
            parts.append(bufs[r][:nr])
        return torch.cat(parts)
    dist.gather(send, dst=dst, group=group)
    return None


def gather_groups(block, height, world, rank, dst=0, group=None):
    """Gather per-rank interleaved 8-row groups (rank r holds rows group_rows(H, world, r),
    packed) into the full [height, W, C] frame on ``dst`` (None elsewhere)."""
    counts = [len(group_rows(height, world, r)) for r in range(world)]
    if block.shape[0] != counts[rank]:
        raise ValueError("rank %d block has %d rows, expected %d" % (rank, block.shape[0], counts[rank]))
    maxrows = max(counts)
    send = block.contiguous()
    if send.shape[0] != maxrows:
        pad = torch.zeros((maxrows,) + tuple(block.shape[1:]), dtype=block.dtype, device=block.device)
        pad[:send.shape[0]] = send
        send = pad
    if rank != dst:
        dist.gather(send, dst=dst, group=group)
        return None
    bufs = [torch.empty_like(send) for _ in range(world)]
    dist.gather(send, gather_list=bufs, dst=dst, group=group)
    frame = torch.empty((height,) + tuple(block.shape[1:]), dtype=block.dtype, device=block.device)
    for r in range(world):
        rows = torch.as_tensor(group_rows(height, world, r), device=block.device)
        frame[rows] = bufs[r][:counts[r]]
    return frame


def render_frame(scene, rank, world, render_rows=None, dtype=torch.float32, dst=0, group=None, interleave=False):
    """Render the whole frame across ``world`` ranks and gather it on ``dst``.

    Contiguous row blocks (default): render_rows(row0, nrows) -> tensor [nrows, W, 3].
    interleave=True: rank r renders the 8-row groups r, r + world, ... (cheap sky rows
    spread over every rank); render_rows(rows) -> tensor [len(rows), W, 3] for the image
    row indices ``rows``. render_rows defaults to the HIP renderer (Scene.render_device)
    on this rank's current GPU. Returns the [H, W, 3] frame (rot90'd reference layout,
    row 0 = top) on ``dst`` and None elsewhere."""
    H = scene.vc.height
    if interleave:
        if render_rows is None:
            block = scene.render_device(groups=(rank, world))
        else:
            block = render_rows(group_rows(H, world, rank))
    else:
        row0, nrows = row_block(H, world, rank)
        if render_rows is None:
            block = scene.render_device(row0=row0, nrows=nrows)
        else:
            block = render_rows(row0, nrows)
    if dtype == torch.uint8 and block.dtype != torch.uint8:
        block = (block.double() * 255.0).to(torch.uint8)  # main.py:327 truncation
    if interleave:
        return gather_groups(block, H, world, rank, dst=dst, group=group)
    return gather_rows(block, H, world, rank, dst=dst, group=group)
