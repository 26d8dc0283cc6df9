"""Hand the RCCL unique id from rank 0 to the other ranks of ONE node without
a second HIP runtime (torch.distributed would map torch's bundled one next to
librtamd.so's).  torchrun (torch.distributed.run) starts every rank of a run
from the same agent process and exports MASTER_PORT / RANK / WORLD_SIZE /
LOCAL_RANK; the id travels through a file in the node's temp directory named
by the port and the agent's pid, written atomically by rank 0.  The
collectives themselves (the frame gather, the bench's max-over-ranks) run
over RCCL inside librtamd.so (rt_dist_*)."""
from __future__ import annotations

import os
import tempfile
import time


def env_ranks() -> tuple[int, int, int]:
    """(rank, world, local_rank) from the launcher's environment (1 process: 0, 1, 0)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def _path(tag: str | None) -> str:
    if tag is None:
        tag = f"{os.environ.get('MASTER_PORT', '0')}_{os.getppid()}"
    return os.path.join(tempfile.gettempdir(), f"rtamd_uid_{tag}")


def share_bytes(rank: int, data: bytes | None, size: int, tag: str | None = None, timeout: float = 300.0) -> bytes:
    """Rank 0 publishes `data` (size bytes); every rank returns it."""
    p = _path(tag)
    if rank == 0:
        assert data is not None and len(data) == size
        tmp = f"{p}.{os.getpid()}.tmp"
        with open(tmp, "wb") as f:
            f.write(data)
        os.replace(tmp, p)
        return data
    t0 = time.monotonic()
    while True:
        try:
            with open(p, "rb") as f:
                got = f.read()
            if len(got) == size:
                return got
        except FileNotFoundError:
            pass
        if time.monotonic() - t0 > timeout:
            raise TimeoutError(f"rank {rank}: no id from rank 0 at {p} after {timeout:.0f} s")
        time.sleep(0.01)


def cleanup(rank: int, tag: str | None = None):
    """Rank 0 removes the id file once every rank holds the communicator."""
    if rank == 0:
        try:
            os.unlink(_path(tag))
        except FileNotFoundError:
            pass
