"""Frame-parallel sharding over the GPUs of one node.

Frames are independent on this path, so N GPUs = N processes (``torch.distributed.run``), each owning a
contiguous slice of the global frame range and its own engine. The only collectives are
  * one broadcast of the packed weight blob from rank 0: ``RcclComm`` + ``Engine.bcast_weights`` on the GPU box
    (the library's own RCCL communicator over xGMI, C ABI ``spef_bcast_weights``), or ``broadcast_blob`` through
    any torch.distributed backend (gloo in the CPU tests),
  * the max-over-ranks of the timed region (bench contract),
  * optionally a gather of the B x 7 pose rows to rank 0 for metrics.
There is nothing to all-reduce. Every function works with any process-group backend, so the CPU gloo tests
exercise exactly the code bench.py runs over RCCL.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist


def world() -> Tuple[int, int]:
    """-> (rank, world_size); (0, 1) when no process group is initialised."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_range(n_frames: int, rank: int, world_size: int) -> Tuple[int, int]:
    """Contiguous [start, stop) slice of ``n_frames`` for ``rank`` (sizes differ by at most one)."""
    base, extra = divmod(n_frames, world_size)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def broadcast_blob(blob: Optional[bytes], device: torch.device, src: int = 0) -> torch.Tensor:
    """Rank ``src`` passes the packed blob, the others ``None``; every rank gets it as a uint8 tensor on
    ``device`` (pass it to ``Engine`` -> ``spef_load_weights_device``: no host round trip on the receivers)."""
    rank, ws = world()
    if rank == src:
        assert blob is not None
        host = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
        n = torch.tensor([host.numel()], dtype=torch.int64, device=device)
    else:
        n = torch.zeros(1, dtype=torch.int64, device=device)
    if ws > 1:
        dist.broadcast(n, src)
    out = torch.empty(int(n.item()), dtype=torch.uint8, device=device)
    if rank == src:
        out.copy_(host)
    if ws > 1:
        dist.broadcast(out, src)
    return out


class RcclComm:
    """An RCCL communicator owned by the SPEF library (``spef_comm_init``), for ``spef_bcast_weights``.

    Rank 0 draws the 128-byte unique id (``spef_comm_unique_id``); the id travels to the other ranks over the
    already-initialised torch.distributed group (``broadcast_object_list``: any backend), the way a C host would ship
    it over MPI or a file. ``int(comm)`` is the ncclComm_t handle. The communicator is nonblocking and every wait on
    it is bounded by ``timeout_ms``: a dead peer makes ``spef_bcast_weights`` abort it (``SpefError`` code
    ``ERR_COMM``) instead of hanging."""

    def __init__(self, device: torch.device, timeout_ms: int = 120_000):
        import ctypes as C
        from . import _lib as L
        self.lib = L.load()
        rank, ws = world()
        idbuf = [None]
        if rank == 0:
            raw = C.create_string_buffer(L.COMM_ID_BYTES)
            L.check(self.lib.spef_comm_unique_id(raw, L.COMM_ID_BYTES))
            idbuf[0] = raw.raw
        if ws > 1:
            dist.broadcast_object_list(idbuf, src=0)
        rid = C.create_string_buffer(bytes(idbuf[0]), L.COMM_ID_BYTES)
        h = C.c_void_p()
        L.check(self.lib.spef_comm_init(torch.device(device).index or 0, ws, rank, rid, int(timeout_ms), C.byref(h)))
        self.handle = h.value

    def __int__(self) -> int:
        return int(self.handle)

    def abort(self) -> None:
        """ncclCommAbort (e.g. when the launcher learns that a peer died); the handle is dead afterwards."""
        if self.handle:
            self.lib.spef_comm_abort(self.handle)

    def close(self) -> None:
        if self.handle:
            self.lib.spef_comm_destroy(self.handle)
            self.handle = None


def max_over_ranks(seconds: float, device: torch.device) -> float:
    """Max of a per-rank wall time (the bench's job time: the slowest rank finishes the job)."""
    _, ws = world()
    if ws == 1:
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_poses(ori: torch.Tensor, pos: torch.Tensor, dst: int = 0):
    """Gather every rank's (ori B_r x 4, pos B_r x 3) to ``dst`` as NumPy arrays in rank order (metrics only).
    Ranks may hold different B_r. Returns (ori, pos) on ``dst``, (None, None) elsewhere."""
    rank, ws = world()
    rows = torch.cat([ori.float(), pos.float()], dim=1).contiguous()
    if ws == 1:
        return rows[:, :4].cpu().numpy(), rows[:, 4:].cpu().numpy()
    n = torch.tensor([rows.shape[0]], dtype=torch.int64, device=rows.device)
    sizes = [torch.zeros_like(n) for _ in range(ws)]
    dist.all_gather(sizes, n)
    m = int(max(int(s.item()) for s in sizes))
    pad = torch.zeros((m, 7), dtype=rows.dtype, device=rows.device)
    pad[:rows.shape[0]] = rows
    bufs = [torch.zeros_like(pad) for _ in range(ws)] if rank == dst else None
    dist.gather(pad, bufs, dst=dst)
    if rank != dst:
        return None, None
    allr = np.concatenate([b[:int(s.item())].cpu().numpy() for b, s in zip(bufs, sizes)], axis=0)
    return allr[:, :4], allr[:, 4:]
