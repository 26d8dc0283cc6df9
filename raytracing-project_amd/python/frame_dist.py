"""Row-strip distribution of one frame over ranks.

Each rank renders interleaved strips of STRIP output rows (strip s goes to rank
s % world), which balances cheap sky rows against expensive geometry rows.
All ranks' row buffers are padded to the same row count so one all_gather
collects them; rank 0 then scatters the real rows into the frame.
Used by bench.py (RCCL, device buffers) and tests/test_dist_gloo.py (gloo).
"""
from __future__ import annotations

STRIP = 8


def strip_rows(H: int, rank: int, world: int, strip: int = STRIP) -> list[int]:
    rows = []
    for s in range((H + strip - 1) // strip):
        if s % world == rank:
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
