"""Row-strip distribution of one frame over ranks.

Each rank renders interleaved strips of STRIP output rows (strip_owners: a
weighted round robin rotated every round, the root lighter), which balances
cheap sky rows against expensive geometry rows.
All ranks' row buffers are padded to the same row count so one all_gather
collects them; rank 0 then scatters the real rows into the frame.

A Python TWIN of the product's partition and chunking (rt_dist.hip
strip_owners / partition_rows / chunk_bounds; tests/test_host_lib.py pins the
partitions equal) for CPU tests and tools only: tests/test_dist_gloo.py runs
it over gloo with the CPU oracle as the renderer.  The product's own rank
protocol (agreements, gathers, placement, failure verdicts) is C++ in
rt_dist.hip dist_frame; bench.py and the CLI go through it (rt_render_dist,
rt_render_multi), and tests/test_gpu_dist_threads.py executes it with
concurrent ranks on one GPU.
"""
from __future__ import annotations

STRIP = 8          # RT_STRIP_ROWS (standard mode)
PAPER_STRIP = 30   # RT_PAPER_STRIP_ROWS (paper mode: + 2 neighbour rows = four 8-row waves)


def strip_for(mode: int) -> int:
    return PAPER_STRIP if mode == 1 else STRIP


ROOT_SHED = {0: 8, 1: 45}   # per mille per rank of the root's weight (rt_dist.hip kRootShedStd / kRootShedPaper)


def strip_owners(n_strips: int, world: int, mode: int = 0, kind: int = 0) -> list[int]:
    """rt_dist.hip strip_owners: smooth weighted round robin over the strips,
    ties to the rank first in a per-round rotation, the root's weight reduced
    by ROOT_SHED[mode] per mille per rank (FP64 output) for its placement work."""
    if world <= 1:
        return [0] * n_strips
    w = [1000] * world
    w[0] = max(500, 1000 - (0 if kind else ROOT_SHED[1 if mode == 1 else 0]) * world)
    total = sum(w)
    cur = [0] * world
    own = []
    for s in range(n_strips):
        for r in range(world):
            cur[r] += w[r]
        rot = (s // world) % world
        best = rot
        for i in range(1, world):
            r = (rot + i) % world
            if cur[r] > cur[best]:
                best = r
        own.append(best)
        cur[best] -= total
    return own


def strip_rows(H: int, rank: int, world: int, strip: int = STRIP, mode: int | None = None, kind: int = 0) -> list[int]:
    """Output rows rank renders (ascending): rt_dist_rows_mode's partition.
    mode defaults to the one whose strip height `strip` is."""
    if mode is None:
        mode = 1 if strip == PAPER_STRIP else 0
    n = (H + strip - 1) // strip
    own = strip_owners(n, world, mode, kind)
    rows = []
    for s in range(n):
        if own[s] == rank:
            rows.extend(range(s * strip, min(H, (s + 1) * strip)))
    return rows


def max_rows(H: int, world: int, strip: int = STRIP) -> int:
    return max(len(strip_rows(H, r, world, strip)) for r in range(world))


def gather_row_index(H: int, world: int, strip: int = STRIP) -> list[int]:
    """Destination row of every slot of the padded all_gather buffer (-1 = pad)."""
    m = max_rows(H, world, strip)
    out = []
    for r in range(world):
        rr = strip_rows(H, r, world, strip)
        out.extend(rr + [-1] * (m - len(rr)))
    return out


def chunk_bounds(m: int, chunks: int, strip: int = 1) -> list[tuple[int, int]]:
    """Split the padded per-rank row list [0, m) into `chunks` contiguous
    pieces of whole strips, of decreasing size (the pipeline units: chunk k is
    gathered while k+1 is traced, so only the smallest, last one's gather is
    exposed; rt_dist.hip chunk_bounds)."""
    units = (m + strip - 1) // strip if m > 0 else 0
    chunks = max(1, min(chunks, units)) if units > 0 else 1
    wsum = chunks * (chunks + 1) // 2   # decreasing sizes: weights chunks, chunks-1, ..., 1
    out, acc = [], 0
    for k in range(chunks):
        u0 = acc * units // wsum
        acc += chunks - k
        u1 = acc * units // wsum
        out.append((min(m, u0 * strip), min(m, u1 * strip)))
    return [(a, b) for a, b in out if b > a] or [(0, 0)]


class DistFrame:
    """One rank's share of a W x H frame and the buffers of its gather.

    rows        output rows this rank renders (interleaved strips)
    mine        [m, W, 3] float64 rows of this rank, padded to m = max_rows
    stage/full  rank 0: [world, m, W, 3] gather target and the [H, W, 3] frame
    slot_rows   rank 0: destination row of every stage slot (-1 = pad)

    run() traces chunk k of `mine` and immediately hands it to an async
    gather to rank 0 (one collective per chunk, on the backend's own stream:
    RCCL over xGMI on the GPU, gloo in the CPU tests), so transfers overlap
    the tracing of later chunks; rank 0 then scatters the slots into `full`.
    With world == 1 `mine` already is the frame (rows 0..H-1 in order)."""

    def __init__(self, W: int, H: int, rank: int, world: int, device, chunks: int = 4, strip: int = STRIP):
        import torch

        self.W, self.H, self.rank, self.world = W, H, rank, world
        self.rows = strip_rows(H, rank, world, strip)
        self.m = max_rows(H, world, strip)
        self.bounds = chunk_bounds(self.m, chunks if world > 1 else 1, strip)
        self.mine = torch.zeros((self.m, W, 3), dtype=torch.float64, device=device)
        self.stage = self.full = self.slot_rows = None
        if world > 1 and rank == 0:
            self.stage = torch.zeros((world, self.m, W, 3), dtype=torch.float64, device=device)
            self.full = torch.zeros((H, W, 3), dtype=torch.float64, device=device)
            self.slot_rows = torch.tensor(gather_row_index(H, world, strip), dtype=torch.int32, device=device)
        elif world == 1:
            self.full = self.mine

    def run(self, trace_chunk, dist=None, scatter=None, streams=None):
        """trace_chunk(a, b, out, stream) renders list entries [a, b) of
        self.rows into out = self.mine[a:b] (may be asynchronous on `stream`);
        scatter(src, slot_rows, full) places gathered slots src[i] at row
        slot_rows[i] of full (rank 0; -1 = padding, skipped).
        With `streams` (torch.cuda.Stream list) chunk k is traced and its
        gather issued on streams[k % len], so consecutive chunks overlap
        their launch tails; the caller joins them (rt_frame_end)."""
        import contextlib

        n = len(self.rows)
        works = []
        for k, (a, b) in enumerate(self.bounds):
            s = streams[k % len(streams)] if streams else None
            hi = min(b, n)
            if hi > a:
                trace_chunk(a, hi, self.mine[a:hi], s)
            if self.world > 1:
                import torch

                gl = [self.stage[r, a:b] for r in range(self.world)] if self.rank == 0 else None
                with torch.cuda.stream(s) if s is not None else contextlib.nullcontext():
                    works.append(dist.gather(self.mine[a:b], gather_list=gl, dst=0, async_op=True))
        # rank 0: place chunk k as soon as its gather is in (the wait orders the
        # current stream after the collective); all but the last chunk's
        # scatter overlap the remaining traces
        for k, w in enumerate(works):
            w.wait()
            if self.rank == 0:
                a, b = self.bounds[k]
                for r in range(self.world):
                    scatter(self.stage[r, a:b], self.slot_rows[r * self.m + a:r * self.m + b], self.full)
        return self.full
