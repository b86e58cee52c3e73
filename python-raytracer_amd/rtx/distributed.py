"""Multi-GPU frame rendering: one process per GPU, each rank renders part of ONE frame, one
gather to rank 0.

The reference parallelises by rendering column strips in separate processes and
stitching them on the filesystem (render.nu:2-23, provided/scene.py:36-37,
provided/main.py:26-28, provided/glue.py:17-27). Here each rank renders on its own GPU
either the row block ``np.array_split(np.arange(H), world)[rank]`` of the final image or
(``interleave=True``, what the bench uses) the 8-row groups rank, rank + world, ...
(``rtx_render_groups``), which spreads the cheap sky rows and the expensive ground rows
over every rank. Camera tables are global and jitter is keyed by the global pixel, so the
frame does not depend on the partition. The rank's rows are converted to the PNG's uint8
on its GPU (``rtx_fb_to_rgb8``: main.py:33's truncation, 4x fewer bytes on the wire) and
gathered to rank 0 with one collective (RCCL over xGMI on MI355X; gloo in the CPU tests),
which puts the rows back in image order with one index_select.
"""
import numpy as np
import torch
import torch.distributed as dist

from .scene import group_rows, split_rows


def row_block(height, world, rank):
    return split_rows(height, world, rank)


def rank_rows(height, world, rank, interleave):
    """Image rows (row 0 = top) rank ``rank`` renders, in its packed order."""
    if interleave:
        return group_rows(height, world, rank)
    r0, n = split_rows(height, world, rank)
    return np.arange(r0, r0 + n)


class FrameGather:
    """The frame's single collective: every rank sends its packed rows (padded to the
    largest rank's count), rank ``dst`` receives them into one buffer and reorders them
    into the [height, W, C] frame. Buffers are allocated once and reused per frame."""

    def __init__(self, height, width, channels, world, rank, dtype, device, interleave=True, dst=0, group=None):
        self.world, self.rank, self.dst, self.group = world, rank, dst, group
        self.rows = [rank_rows(height, world, r, interleave) for r in range(world)]
        self.nrows = len(self.rows[rank])
        self.maxrows = max(len(r) for r in self.rows)
        shape = (self.maxrows, width, channels)
        self.send = torch.zeros(shape, dtype=dtype, device=device)
        self.block = self.send[:self.nrows]  # this rank renders (or converts) into it
        if rank == dst:
            self.recv = torch.empty((world,) + shape, dtype=dtype, device=device)
            self.recv_list = list(self.recv.unbind(0))
            src = np.empty(height, np.int64)  # frame row -> row of recv viewed as [world * maxrows]
            for r, rows in enumerate(self.rows):
                src[rows] = r * self.maxrows + np.arange(len(rows))
            self.index = torch.as_tensor(src, device=device)

    def __call__(self):
        """Gather the ranks' blocks; returns the frame on ``dst`` and None elsewhere."""
        if self.rank != self.dst:
            dist.gather(self.send, dst=self.dst, group=self.group)
            return None
        dist.gather(self.send, gather_list=self.recv_list, dst=self.dst, group=self.group)
        flat = self.recv.view((self.world * self.maxrows,) + tuple(self.recv.shape[2:]))
        return torch.index_select(flat, 0, self.index)


def gather_rows(block, height, world, rank, dst=0, group=None, interleave=False):
    """Gather per-rank packed row blocks [nrows_r, W, C] into the full [height, W, C] frame
    on ``dst`` (None on other ranks). Any dtype/device the backend takes."""
    g = FrameGather(height, block.shape[1], block.shape[2], world, rank, block.dtype, block.device,
                    interleave=interleave, dst=dst, group=group)
    if block.shape[0] != g.nrows:
        raise ValueError("rank %d block has %d rows, expected %d" % (rank, block.shape[0], g.nrows))
    g.block.copy_(block)
    return g()


def gather_groups(block, height, world, rank, dst=0, group=None):
    """gather_rows for interleaved 8-row groups (rank r holds group_rows(H, world, r))."""
    return gather_rows(block, height, world, rank, dst=dst, group=group, interleave=True)


def to_rgb8(block):
    """(block * 255.0) truncated to uint8 (main.py:33): rtx_fb_to_rgb8 on the rank's GPU.
    CPU blocks (the gloo tests' host emulation of a rank) are converted with the same
    fp64 multiply and truncation on the host."""
    if block.is_cuda:
        from .scene import fb_to_rgb8
        return fb_to_rgb8(block)
    return torch.from_numpy((block.numpy().astype(np.float64) * 255.0).astype(np.uint8))


def render_frame(scene, rank, world, render_rows=None, dtype=torch.float32, dst=0, group=None, interleave=False):
    """Render the whole frame across ``world`` ranks and gather it on ``dst``.

    Contiguous row blocks (default): render_rows(row0, nrows) -> tensor [nrows, W, 3].
    interleave=True: rank r renders the 8-row groups r, r + world, ...; render_rows(rows)
    -> tensor [len(rows), W, 3] for the image row indices ``rows``. render_rows defaults
    to the HIP renderer (Scene.render_device) on this rank's current GPU. Returns the
    [H, W, 3] frame (rot90'd reference layout, row 0 = top) on ``dst``, None elsewhere."""
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
        block = to_rgb8(block)
    return gather_rows(block, H, world, rank, dst=dst, group=group, interleave=interleave)
