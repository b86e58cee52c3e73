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
        # contiguous equal blocks (np.array_split with world | height) arrive in image order:
        # the receive buffer IS the frame, no reorder
        self.in_order = not interleave and height == world * self.maxrows
        if rank == dst:
            self.recv = torch.empty((world,) + shape, dtype=dtype, device=device)
            self.recv_list = list(self.recv.unbind(0))
            src = np.empty(height, np.int64)  # frame row -> row of recv viewed as [world * maxrows]
            for r, rows in enumerate(self.rows):
                src[rows] = r * self.maxrows + np.arange(len(rows))
            self.index = torch.as_tensor(src, device=device)

    def frame(self):
        """The gathered frame [height, W, C] on ``dst`` (after the gather completed)."""
        flat = self.recv.view((self.world * self.maxrows,) + tuple(self.recv.shape[2:]))
        return flat if self.in_order else torch.index_select(flat, 0, self.index)

    def __call__(self):
        """Gather the ranks' blocks; returns the frame on ``dst`` and None elsewhere."""
        if self.rank != self.dst:
            dist.gather(self.send, dst=self.dst, group=self.group)
            return None
        dist.gather(self.send, gather_list=self.recv_list, dst=self.dst, group=self.group)
        return self.frame()


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
    fp64 multiply and truncation on the host. (The bench's pipeline renders uint8
    directly: rtx_render_groups_rgb8.)"""
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


class FramePipeline:
    """The multi-GPU frame loop of bench.py (north star: one frame sharded across the node,
    one gather at the end): every step renders this rank's rows of the next frame straight
    into uint8 (rtx_render_rgb8 / rtx_render_groups_rgb8: main.py:33's conversion fused
    into the render kernel) and starts their gather to ``dst`` asynchronously; the previous
    frame's gather is then awaited (a stream wait, not a host wait, on RCCL). Two buffer
    slots, so frame k's gather runs while frame k + 1 renders.

    Partition: ``interleave=True`` gives rank r the 8-row groups r, r + N, ... (balances
    cheap sky rows against expensive ground rows; rank 0 reorders the gathered rows with
    one index_select); ``interleave=False`` the np.array_split row blocks, which for
    N | height arrive in image order (zero-copy frame). Default: interleave when a pixel
    has several samples (render time dominates), blocks for 1-spp frames (the gather
    dominates). ``render_block(out, rows)`` fills this rank's uint8 rows [len(rows), W, 3];
    the CPU tests inject the host emulation."""

    def __init__(self, scene, rank, world, dst=0, group=None, device=None, render_block=None, interleave=None):
        H, W = scene.vc.height, scene.vc.width
        device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        if interleave is None:
            interleave = scene.samples_per_pixel > 1
        self.rank, self.dst, self.group, self.interleave = rank, dst, group, interleave
        self.slots = [FrameGather(H, W, 3, world, rank, torch.uint8, device, interleave=interleave, dst=dst,
                                  group=group) for _ in range(2)]
        self.rows = self.slots[0].rows[rank]
        if render_block is None:
            if interleave:
                def render_block(out, rows):
                    scene.render_device(groups=(rank, world), out=out)
            else:
                r0, n = row_block(H, world, rank)

                def render_block(out, rows):
                    scene.render_device(row0=r0, nrows=n, out=out)
        self.render_block = render_block
        self.k = 0
        self.prev = None  # (work, slot) of the last submitted frame

    def _finish(self, work, slot):
        work.wait()
        return slot.frame() if self.rank == self.dst else None

    def render(self):
        """Render this rank's rows of the next frame into the free slot."""
        slot = self.slots[self.k % 2]
        if slot.nrows:
            self.render_block(slot.block, self.rows)
        return slot

    def step(self):
        """Submit the next frame; returns the previous frame on ``dst`` (None elsewhere and
        on the first step)."""
        slot = self.render()
        if self.rank == self.dst:
            work = dist.gather(slot.send, gather_list=slot.recv_list, dst=self.dst, group=self.group, async_op=True)
        else:
            work = dist.gather(slot.send, dst=self.dst, group=self.group, async_op=True)
        prev, self.prev = self.prev, (work, slot)
        self.k += 1
        return self._finish(*prev) if prev is not None else None

    def flush(self):
        """Wait for the last submitted frame; returns it on ``dst``."""
        prev, self.prev = self.prev, None
        return self._finish(*prev) if prev is not None else None
