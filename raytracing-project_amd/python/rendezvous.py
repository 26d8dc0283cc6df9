"""Hand the RCCL unique id from rank 0 to the other ranks of ONE node without
a second HIP runtime (torch.distributed would map torch's bundled one next to
librtamd.so's).  torchrun (torch.distributed.run) starts every rank of a run
from the same agent process and exports MASTER_PORT / RANK / WORLD_SIZE /
LOCAL_RANK (bench.py --gpus N without a launcher spawns its ranks the same
way); the id travels through an owner-only file in the node's temp directory
named by the port and the launcher's run id, written atomically by rank 0.  The
collectives themselves (the frame gather, the bench's max-over-ranks) run
over RCCL inside librtamd.so (rt_dist_*)."""
from __future__ import annotations

import os
import tempfile
import time


def env_ranks() -> tuple[int, int, int]:
    """(rank, world, local_rank) from the launcher's environment (1 process: 0, 1, 0).

    The id file only reaches ranks on this node, so a job whose ranks span
    nodes (WORLD_SIZE != LOCAL_WORLD_SIZE) is refused here instead of timing
    out in share_bytes."""
    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if world != local_world:
        raise RuntimeError(f"rendezvous: WORLD_SIZE={world} but LOCAL_WORLD_SIZE={local_world}: the RCCL id is "
                           "handed over through a node-local file, so every rank must run on this node")
    return rank, world, int(os.environ.get("LOCAL_RANK", "0"))


def _path(tag: str | None) -> str:
    if tag is None:
        # port + the launcher's run id when it has a real one (torchrun:
        # TORCHELASTIC_RUN_ID, which static rendezvous leaves at "none";
        # bench.py: a unique RTAMD_RUN_ID per run), so ranks started through
        # their own wrapper processes (a per-rank shell or numactl wrapper,
        # per-task srun) still meet.  Only without a real run id does the
        # common parent (the launcher's agent) stand in for it, so a file left
        # by a run that died before cleanup() is never read by the next run.
        run = os.environ.get("RTAMD_RUN_ID") or os.environ.get("TORCHELASTIC_RUN_ID") or ""
        if run.strip().lower() in ("", "none"):
            run = f"ppid{os.getppid()}"
        tag = f"{os.environ.get('MASTER_PORT', '0')}_{run}"
    return os.path.join(tempfile.gettempdir(), f"rtamd_uid_{tag}")


def share_bytes(rank: int, data: bytes | None, size: int, tag: str | None = None, timeout: float = 300.0) -> bytes:
    """Rank 0 publishes `data` (size bytes); every rank returns it.  The file
    is created owner-only (0600): it holds the communicator's unique id."""
    p = _path(tag)
    if rank == 0:
        assert data is not None and len(data) == size
        tmp = f"{p}.{os.getpid()}.tmp"
        fd = os.open(tmp, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
        with os.fdopen(fd, "wb") as f:
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
