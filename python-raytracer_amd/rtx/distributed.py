"""Multi-GPU frame rendering: one process per GPU, each rank renders part of ONE frame, one
gather of that frame to one rank (rank 0, or the frame's owner in FrameExchange).

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
import ctypes

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
    into the [height, W, C] frame. Buffers are allocated once and reused per frame.
    ``dst`` renders its own rows in place, into its slot of the receive buffer, and hands
    that very tensor to the gather as its input (the collective's root copy is then a
    no-op: ``copy_`` of a tensor onto itself); one rank needs no collective at all."""

    def __init__(self, height, width, channels, world, rank, dtype, device, interleave=True, dst=0, group=None):
        self.world, self.rank, self.dst, self.group = world, rank, dst, group
        self.rows = [rank_rows(height, world, r, interleave) for r in range(world)]
        self.nrows = len(self.rows[rank])
        self.maxrows = max(len(r) for r in self.rows)
        self.height = height
        shape = (self.maxrows, width, channels)
        # contiguous equal blocks (np.array_split with world | height) arrive in image order:
        # the receive buffer IS the frame, no reorder
        self.in_order = not interleave and height == world * self.maxrows
        if rank == dst:
            self.recv = torch.zeros((world,) + shape, dtype=dtype, device=device)
            self.recv_list = list(self.recv.unbind(0))
            self.send = self.recv_list[dst]
            src = np.empty(height, np.int64)  # frame row -> row of recv viewed as [world * maxrows]
            for r, rows in enumerate(self.rows):
                src[rows] = r * self.maxrows + np.arange(len(rows))
            self.in_order = self.in_order or bool(np.array_equal(src, np.arange(height)))
            self.index = torch.as_tensor(src, device=device)
        else:
            self.send = torch.zeros(shape, dtype=dtype, device=device)
        self.block = self.send[:self.nrows]  # this rank renders (or converts) into it

    def frame(self):
        """The gathered frame [height, W, C] on ``dst`` (after the gather completed); a view
        of the receive buffer when the rows arrive in image order (valid until the buffer's
        next gather), else a new tensor."""
        flat = self.recv.view((self.world * self.maxrows,) + tuple(self.recv.shape[2:]))
        return flat[:self.height] if self.in_order else torch.index_select(flat, 0, self.index)

    def start(self, async_op=False):
        """Issue the gather (None at world 1: nothing to move)."""
        if self.world == 1:
            return None
        if self.rank != self.dst:
            return dist.gather(self.send, dst=self.dst, group=self.group, async_op=async_op)
        return dist.gather(self.send, gather_list=self.recv_list, dst=self.dst, group=self.group, async_op=async_op)

    def __call__(self):
        """Gather the ranks' blocks; returns the frame on ``dst`` and None elsewhere."""
        self.start()
        return self.frame() if self.rank == self.dst else None


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


class BlockGather:
    """A frame gathered to rank 0 from uneven contiguous row blocks: rank 0 renders rows
    [0, root_rows) in place, the other ranks split the rest with np.array_split and send
    their blocks to rank 0 in ONE all_to_all_single with uneven splits (each rank's rows
    straight to rank 0, nothing elsewhere), landing in image order -- rank 0's buffer IS
    the frame. Rank 0's own rows cross no link, so giving it more of them balances the
    render against the other ranks' transfer into rank 0 (FrameGraph ``root_rows``;
    bench.py tunes the share)."""

    def __init__(self, height, width, world, rank, device, root_rows, group=None):
        x = int(root_rows)
        if world < 2 or not 0 < x < height:
            raise ValueError("root_rows must leave rows to every rank: 0 < %d < %d, world >= 2" % (x, height))
        self.world, self.rank, self.dst, self.group = world, rank, 0, group
        rest = [x + b for b in np.array_split(np.arange(height - x), world - 1)]
        self.rows = [np.arange(0, x)] + rest
        self.nrows = len(self.rows[rank])
        self.height, self.in_order = height, True
        if rank == 0:
            self.frame_buf = torch.zeros((height, width, 3), dtype=torch.uint8, device=device)
            self.block = self.frame_buf[:x]
            self.send = self.frame_buf[:0]
            self.recv = self.frame_buf[x:]
            self.in_splits, self.out_splits = [0] * world, [0] + [len(r) for r in rest]
        else:
            self.send = torch.zeros((self.nrows, width, 3), dtype=torch.uint8, device=device)
            self.block = self.send
            self.recv = torch.empty((0, width, 3), dtype=torch.uint8, device=device)
            self.in_splits, self.out_splits = [self.nrows if j == 0 else 0 for j in range(world)], [0] * world

    def start(self, async_op=False):
        return dist.all_to_all_single(self.recv, self.send, output_split_sizes=self.out_splits,
                                      input_split_sizes=self.in_splits, group=self.group, async_op=async_op)

    def frame(self):
        return self.frame_buf


class FrameGraph:
    """ONE frame sharded over the ranks per step, gathered to ``dst`` and awaited before the
    next step (bench.py's N > 1 value; the reference's strip renders + glue,
    render.nu:10-15, provided/glue.py:17-27), issued without per-frame Python: this rank's
    render of its rows (uint8, main.py:33's conversion fused), the RCCL gather
    (FrameGather) and, on ``dst``, the reorder into image order are recorded ONCE as a HIP
    graph and replayed per frame -- ``step()`` is one graph launch; ``run(n)`` launches n
    frames from C (rtx_graph_launch), ``frames_per_graph`` of them per graph: a second graph
    records that many frames one after the other (each still rendered, gathered and
    reordered in stream order before the next), so a frame costs 1 / frames_per_graph of
    a hipGraphLaunch of host time (~4.6 us per launch on the MI355X box, profiles/r06/s2).

    Partition: contiguous np.array_split row blocks for one-sample frames (``interleave``
    None and samples_per_pixel == 1): with N | H they arrive in image order and the gathered
    buffer IS the frame; interleaved 8-row groups otherwise (render-bound multi-sample
    frames balance better), put in order by an index_select recorded into the graph.
    ``root_rows`` (blocks, N > 1, dst 0): rank 0 renders that many rows itself and the
    others split the rest (BlockGather: one all_to_all_single with uneven splits).

    The graph bakes in the scene's device buffers: it is recorded again when the scene's
    upload generation changes (a camera upload or an edit re-upload, checked per ``step``;
    ``run`` checks once). ``graph=False`` (or a CPU device: the gloo tests' host
    emulation) issues the same three steps eagerly. ``collective_at_one``: issue the
    (one-rank) gather even at world 1, so a one-rank group records RCCL's calls too
    (tests/test_gpu_frame_loop.py); otherwise world 1 has no collective at all.
    ``render_block(out, rows)`` fills this rank's rows (uint8 [len(rows), W, 3], image rows
    ``rows``) -- the CPU tests inject the host emulation."""

    def __init__(self, scene, rank, world, dst=0, group=None, device=None, interleave=None, render_block=None,
                 graph=True, collective_at_one=False, frames_per_graph=8, root_rows=None):
        H, W = scene.vc.height, scene.vc.width
        device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        if interleave is None:
            interleave = scene.samples_per_pixel > 1
        self.scene, self.rank, self.world, self.dst, self.interleave = scene, rank, world, dst, interleave
        self.root_rows = None
        if root_rows is not None and not interleave and world > 1 and dst == 0:
            self.root_rows = int(root_rows)
            self.g = BlockGather(H, W, world, rank, device, self.root_rows, group=group)
        else:
            self.g = FrameGather(H, W, 3, world, rank, torch.uint8, device, interleave=interleave, dst=dst, group=group)
        self.rows = self.g.rows[rank]
        self.collective = world > 1 or collective_at_one
        self.out = None
        if rank == dst and not self.g.in_order:
            self.out = torch.empty((H, W, 3), dtype=torch.uint8, device=device)
        if render_block is None:
            if interleave:
                def render_block(out, rows):
                    scene.render_device(groups=(rank, world), out=out)
            else:
                def render_block(out, rows):
                    scene.render_device(row0=int(rows[0]), nrows=len(rows), out=out)
        self.render_block = render_block
        self.graph_on = graph and device.type == "cuda"
        self.kmax = max(1, int(frames_per_graph))
        self.graph = None   # one frame
        self.graphk = None  # kmax frames
        self._state = None

    def _issue(self):
        """The frame's three steps, in stream order on the current stream."""
        g = self.g
        if g.nrows:
            self.render_block(g.block, self.rows)
        if isinstance(g, BlockGather):
            g.start()
        elif self.collective:
            if self.rank != self.dst:
                dist.gather(g.send, dst=self.dst, group=g.group)
            else:
                dist.gather(g.send, gather_list=g.recv_list, dst=self.dst, group=g.group)
        if self.out is not None:
            flat = g.recv.view((g.world * g.maxrows,) + tuple(g.recv.shape[2:]))
            torch.index_select(flat, 0, g.index, out=self.out)

    def _scene_state(self):
        sc = self.scene
        if hasattr(sc, "_set_camera"):  # a changed camera or scene is uploaded (new tables) first
            sc._set_camera(0, 1)
        return getattr(sc, "_gen", None)

    def capture(self):
        """Record the frame as a HIP graph: the specialized kernels are compiled and the
        frame issued eagerly first (allocations, the tile schedule's measuring frames), then
        recorded without executing. Scenes whose uint8 renders run the generic kernels
        (which stage through a library scratch buffer) stay eager."""
        if hasattr(self.scene, "jit_wait"):
            self._issue()
            self.scene.jit_wait()
        for _ in range(3):
            self._issue()
        torch.cuda.synchronize()
        self._state = self._scene_state()
        if self.g.nrows and not getattr(self.scene, "last_kernel", "rtx_jit_render_").startswith("rtx_jit_render_"):
            self.graph_on = False
            self.graph = None
            return
        ref = self.frame().clone() if self.rank == self.dst else None
        gr = gk = None
        ok, why = True, ""
        try:
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, capture_error_mode="thread_local"):
                self._issue()
            if self.kmax > 1:
                gk = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gk, capture_error_mode="thread_local"):
                    for _ in range(self.kmax):
                        self._issue()
            torch.cuda.synchronize()
        except Exception as e:  # noqa: BLE001 -- a backend that cannot record its collective
            ok, why = False, "capture failed on rank %d: %r" % (self.rank, e)
        ok = self._agree(ok)  # (every rank records, or none: the frame loop stays eager)
        if ok:
            # one replay of each graph, which must finish and deliver the eager frame's bytes
            for g in (gr, gk):
                if g is not None:
                    self._replay_checked(g)
            same = True if ref is None else bool(torch.equal(self.frame(), ref))
            ok = self._agree(same)
            if not ok:
                why = "a replayed frame differs from the eager frame"
        if not ok:
            import warnings
            warnings.warn("FrameGraph: issuing frames eagerly (%s)" % (why or "another rank could not record"))
            self.graph_on = False
            self.graph = self.graphk = None
            return
        self.graph, self.graphk = gr, gk

    def _agree(self, ok):
        """Whether every rank's ok holds (an all_reduce, outside any capture)."""
        if not (self.collective and dist.is_available() and dist.is_initialized()):
            return ok
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=self.g.send.device)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.g.group)
        return bool(t.item())

    @staticmethod
    def _replay_checked(g, timeout_s=60.0):
        """Replay g once and wait for it, bounded: a collective that never completes inside
        a graph raises instead of hanging the frame loop."""
        import time
        ev = torch.cuda.Event()
        g.replay()
        ev.record()
        t0 = time.perf_counter()
        while not ev.query():
            if time.perf_counter() - t0 > timeout_s:
                raise RuntimeError("FrameGraph: a replayed frame did not complete in %.0f s" % timeout_s)
            time.sleep(1e-4)

    def step(self):
        """Issue one frame (asynchronous; frames are stream-ordered, so each one's gather is
        complete before the next frame's render writes the buffers)."""
        if not self.graph_on:
            self._issue()
            return
        if self.graph is None or self._scene_state() != self._state:
            self.capture()
            if not self.graph_on:
                self._issue()
                return
        self.graph.replay()

    def run(self, n, stream=None):
        """Issue n frames: rtx_graph_launch calls (n / frames_per_graph launches of the
        multi-frame graph, then the rest one frame each) when the frame is a graph, else n
        eager frames."""
        if n <= 0:
            return
        if self.graph_on and (self.graph is None or self._scene_state() != self._state):
            self.capture()
        if not self.graph_on:
            for _ in range(n):
                self._issue()
            return
        from . import _native as N
        st = ctypes.c_void_p((stream if stream is not None else torch.cuda.current_stream()).cuda_stream)
        q, r = divmod(int(n), self.kmax) if self.graphk is not None else (0, int(n))
        if q:
            N.call("rtx_graph_launch", ctypes.c_void_p(self.graphk.raw_cuda_graph_exec()), q, st)
        if r:
            N.call("rtx_graph_launch", ctypes.c_void_p(self.graph.raw_cuda_graph_exec()), r, st)

    def frame(self):
        """The last frame on ``dst`` ([H, W, 3] uint8, valid until the next step), None
        elsewhere. Synchronize the stream first to read it."""
        if self.rank != self.dst:
            return None
        return self.out if self.out is not None else self.g.frame()


class FramePipeline:
    """Every frame sharded across the node and gathered to ``dst`` (bench.py reports it
    beside FrameExchange, its N > 1 headline, as "gather_to_rank0"): every step renders this rank's rows of the next frame straight
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
    the CPU tests inject the host emulation. A returned frame is a view of a slot's
    receive buffer when its rows arrive in image order (always at N = 1), valid until that
    slot is gathered again two steps later -- clone it to keep it."""

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
        if work is not None:
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
        work = slot.start(async_op=True)
        prev, self.prev = self.prev, (work, slot)
        self.k += 1
        return self._finish(*prev) if prev is not None else None

    def flush(self):
        """Wait for the last submitted frame; returns it on ``dst``."""
        prev, self.prev = self.prev, None
        return self._finish(*prev) if prev is not None else None


class FrameExchange:
    """The multi-GPU frame loop of bench.py at N > 1: every frame is sharded over the N
    ranks and gathered to ONE rank, its owner -- frame k belongs to rank k mod N, the
    process that would write its PNG (the reference writes each strip's file from its own
    process and glues them: provided/main.py:26-28, provided/glue.py:17-27).

    FramePipeline gathers every frame to rank 0, so the frame rate is capped by rank 0's
    ingress: (N - 1) / N of every frame over its links, while the other ranks' links idle.
    Here the gathers of N consecutive frames (frame j of a group to rank j) are issued as
    one ``all_to_all_single``: each rank sends its rows of frame j straight to rank j, so
    every xGMI link of the full mesh carries 1 / N of a frame per group and the exchange
    costs ~1 / N of a gather per frame.

    No rank sends anything to itself: its rows of its OWN frame are rendered straight into
    the place where the owner assembles that frame, and the collective's split sizes are 0
    for the rank itself. Per group buffer, one allocation Z of 2N - 1 row slots
    [maxrows, W, 3]:

        Z[0 : N-1]    this rank's rows of the peers' frames, frame j at slot p(j)
                      (p(j) = j for j < rank, j - 1 above): the collective's input
        Z[N-1]        this rank's rows of its own frame
        Z[N : 2N-1]   the peers' rows of this rank's frame, from rank s at N + p(s):
                      the collective's output

    so Z[N-1 : 2N-1] holds the owner's whole frame ([N * maxrows] rows) and one
    index_select puts it in image order. At N = 1 there is no collective at all and the
    frame is Z[0] itself.

    Frames are submitted one per ``step``; a group is rendered once its N frames are
    submitted (this rank's rows of each, uint8, fused), then its exchange starts
    asynchronously and the previous group's exchange is awaited (a stream wait on RCCL), so
    an exchange overlaps the next group's renders. Two group buffers. With the default
    renderer a full group is ONE launch (``Scene.render_frames``: gridDim.y = N frames into
    Z[0 : N], all of one scene state -- the bench's static frame), which both keeps the
    host ahead (a Python render call costs ~9 us of host time, a 1/8-frame render ~3.5 us
    of GPU time) and fills the GPU that one 1/N-frame launch leaves partly idle. Otherwise
    ``graph=True`` records the N renders of each buffer once as a HIP graph and replays it
    per group (needs a render_block that does not depend on k, like the bench's static
    frame; the scene's camera is re-checked per group and the graphs are re-recorded when
    its upload or device state changed; scenes that run the generic kernels stay eager). ``flush``
    renders and exchanges a partial last group (uneven splits: no rows for the frames that
    were not submitted).

    ``render_block(out, rows, k)`` fills this rank's uint8 rows [len(rows), W, 3] of frame
    k (the CPU tests inject the host emulation). ``step`` and ``flush`` return the list
    of (k, frame [H, W, 3]) this rank owns that completed; a frame is a new tensor, except
    when the rows already arrive in image order (N = 1, or rank 0 of some partitions):
    then it is a view of a group buffer, valid until that buffer is rendered again (two
    groups later) -- clone it to keep it."""

    def __init__(self, scene, rank, world, group=None, device=None, render_block=None, interleave=True, graph=False):
        H, W = scene.vc.height, scene.vc.width
        device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.scene, self.rank, self.world, self.group, self.interleave = scene, rank, world, group, interleave
        self.rows_all = [rank_rows(H, world, r, interleave) for r in range(world)]
        self.rows = self.rows_all[rank]
        self.nrows = len(self.rows)
        self.maxrows = max(len(r) for r in self.rows_all)
        N = world
        self.Z = [torch.zeros((2 * N - 1, self.maxrows, W, 3), dtype=torch.uint8, device=device) for _ in range(2)]
        pos = np.empty(H, np.int64)  # frame row -> row of Z[N-1:] viewed as [N * maxrows]
        for s, rws in enumerate(self.rows_all):
            base = 0 if s == rank else (1 + self._peer(s)) * self.maxrows
            pos[rws] = base + np.arange(len(rws))
        # rows already in image order (N = 1, and the first rank of some partitions): the
        # frame is a view of Z[N-1:]
        self.identity = bool(np.array_equal(pos, np.arange(H)))
        self.H = H
        self.index = torch.as_tensor(pos, device=device)
        # the default renderer renders a group in ONE launch (rtx_render_frames /
        # rtx_render_groups_frames)
        self.render_frames = None
        if render_block is None:
            if interleave:
                def render_block(out, rows, k):
                    scene.render_device(groups=(rank, world), out=out)

                def render_frames(out):
                    scene.render_frames(out, groups=(rank, world))
            else:
                r0, n = row_block(H, world, rank)

                def render_block(out, rows, k):
                    scene.render_device(row0=r0, nrows=n, out=out)

                def render_frames(out):
                    scene.render_frames(out, row0=r0, nrows=n)
            self.render_frames = render_frames
        self.render_block = render_block
        self.graph = graph and device.type == "cuda" and self.render_frames is None
        self.graphs = [None, None]
        self._graph_state = None
        self.k = 0
        self.pending = None  # (work, buffer, first frame index, frames) of the last exchange

    def _peer(self, j):
        """Slot of peer j among this rank's N - 1 peer slots."""
        return j if j < self.rank else j - 1

    def slot(self, buf, j):
        """Where this rank renders its rows of frame j of a group (uint8 [nrows, W, 3])."""
        i = self.world - 1 if j == self.rank else self._peer(j)
        return self.Z[buf][i, :self.nrows]

    def render_group(self, buf, first, nframes):
        """Render this rank's rows of frames first .. first + nframes - 1 of a group into
        their slots of buffer ``buf`` (a graph replay for a full group in graph mode)."""
        if not self.nrows:
            return
        if self.render_frames is not None:  # one scene state: N interchangeable frames, one launch
            self.render_frames(self.Z[buf][:self.world])
            return
        if self.graph and nframes == self.world:
            if hasattr(self.scene, "_set_camera"):  # a changed camera is uploaded (new tables) first
                self.scene._set_camera(0, 1)
            if self.graphs[buf] is None or self._graph_state != self._state():
                self.capture(buf)
            if self.graph:
                self.graphs[buf].replay()
                return
        for j in range(nframes):
            self.render_block(self.slot(buf, j), self.rows, first + j)

    def _state(self):
        """What a captured graph bakes in: the scene's device handle and camera upload,
        named by the scene's upload generation (rtx.Scene counts every native re-create and
        camera upload from a process-wide counter, so a freed and re-allocated handle or
        table never matches a recorded state)."""
        sc = self.scene
        gen = getattr(sc, "_gen", None)
        if gen is not None:
            return gen
        nat = getattr(sc, "_native", None)  # scenes of other types: identities
        return (id(nat), getattr(nat, "h", None) and nat.h.value, id(getattr(sc, "_cam_info", None)))

    def capture(self, buf):
        """Record both buffers' group renders as HIP graphs (graph mode), rendering buffer
        ``buf`` (the one about to be rendered; the other may hold a frame not yet
        delivered) eagerly first, which compiles any specialized kernel. The capture is
        thread-local (the process group's watchdog thread keeps querying its events
        meanwhile) and records without executing, so an exchange in flight is untouched."""
        if not self.nrows:
            return
        for j in range(self.world):
            self.render_block(self.slot(buf, j), self.rows, j)
        if hasattr(self.scene, "jit_wait"):  # the specialized kernels (compiling on a host thread)
            self.scene.jit_wait()
            for j in range(self.world):
                self.render_block(self.slot(buf, j), self.rows, j)
        torch.cuda.synchronize()
        if not getattr(self.scene, "last_kernel", "rtx_jit_render_").startswith("rtx_jit_render_"):
            # the generic kernels' uint8 renders stage through a library scratch buffer that
            # a larger render may reallocate under a recorded graph: stay eager
            self.graph = False
            self.graphs = [None, None]
            return
        for buf in (0, 1):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                for j in range(self.world):
                    self.render_block(self.slot(buf, j), self.rows, j)
            self.graphs[buf] = g
        torch.cuda.synchronize()
        self._graph_state = self._state()

    def render(self):
        """One frame's render alone (bench.py's breakdown; not part of the frame loop)."""
        if self.nrows:
            self.render_block(self.slot(0, self.rank), self.rows, 0)

    def _frame(self, buf):
        flat = self.Z[buf][self.world - 1:].reshape((self.world * self.maxrows,) + tuple(self.Z[buf].shape[2:]))
        return flat[:self.H] if self.identity else torch.index_select(flat, 0, self.index)

    def _exchange(self, buf, nframes, async_op=True):
        """frame j's rows to rank j, for the group's first nframes frames; no self-sends."""
        N, m = self.world, self.maxrows
        if N == 1:
            return None
        Z = self.Z[buf]
        ins = [m if (j < nframes and j != self.rank) else 0 for j in range(N)]
        outs = [m if (self.rank < nframes and s != self.rank) else 0 for s in range(N)]
        flat = Z.view((Z.shape[0] * m,) + tuple(Z.shape[2:]))
        send = flat[:sum(ins)]
        recv = flat[N * m:N * m + sum(outs)]
        return dist.all_to_all_single(recv, send, output_split_sizes=outs, input_split_sizes=ins, group=self.group,
                                      async_op=async_op)

    def _submit_group(self, nframes):
        """Render the group that ends at frame k - 1 (nframes of it) and start its one
        collective. Returns the previous group's frames."""
        first = self.k - nframes
        buf = (first // self.world) % 2
        self.render_group(buf, first, nframes)
        work = self._exchange(buf, nframes)
        prev, self.pending = self.pending, (work, buf, first, nframes)
        return self._finish(prev)

    def _finish(self, pending):
        if pending is None:
            return []
        work, buf, first, nframes = pending
        if work is not None:
            work.wait()
        return [(first + self.rank, self._frame(buf))] if self.rank < nframes else []

    def exchange_once(self):
        """One full-group exchange of buffer 0, awaited (a stream wait): its cost alone
        (bench.py's breakdown; not part of the frame loop). Nothing at N = 1."""
        work = self._exchange(0, self.world)
        if work is not None:
            work.wait()

    def step(self):
        """Submit the next frame; returns this rank's completed frames (see the class)."""
        self.k += 1
        return self._submit_group(self.world) if self.k % self.world == 0 else []

    def flush(self):
        """Render and exchange a partial last group, and wait for everything submitted."""
        out = []
        j = self.k % self.world
        if j:
            out += self._submit_group(j)
        pending, self.pending = self.pending, None
        return out + self._finish(pending)
