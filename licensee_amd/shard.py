"""Multi-GPU sharding of the Dice path (one process per GPU, torch.distributed).

Files are independent and templates are read-only, so each rank scores a
contiguous, disjoint shard with its own replicated template context -- no data-path
collective. Only the 16-byte per-file results move, once, after scoring:

  * ``host``       -- every rank copies its results (D2H) straight into its slice of a
                      node-shared host buffer that rank 0 owns (``SharedResults``): after one
                      barrier rank 0 holds every result;
  * ``collective`` -- results are packed into one int32 [n, 4] tensor per rank
                      (best, overlap, score as two int32 words) and gathered to rank 0 (RCCL
                      over xGMI with the nccl backend, gloo on CPU), then copied to rank 0's host.

Both end with the whole job's results in rank 0's host memory; bench.py times both and reports
the faster one; tests/test_distributed.py runs both with gloo at world size 2.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np


def shard_range(rank: int, world: int, files_per_rank: int) -> Tuple[int, int]:
    """Weak scaling: rank r owns global files [r*F, (r+1)*F)."""
    if not (0 <= rank < world) or files_per_rank < 0:
        raise ValueError('bad shard arguments')
    return rank * files_per_rank, files_per_rank


def pack_results(best: np.ndarray, overlap: np.ndarray, score: np.ndarray) -> np.ndarray:
    """(int32 best, uint32 overlap, float64 score) -> int32 [n, 4] (bit-preserving)."""
    n = best.shape[0]
    out = np.empty((n, 4), np.int32)
    out[:, 0] = best
    out[:, 1] = overlap.view(np.int32)
    out[:, 2:4] = np.ascontiguousarray(score, np.float64).view(np.int32).reshape(n, 2)
    return out


def unpack_results(packed: np.ndarray):
    packed = np.ascontiguousarray(packed, np.int32)
    best = packed[:, 0].copy()
    overlap = packed[:, 1].copy().view(np.uint32)
    score = np.ascontiguousarray(packed[:, 2:4]).view(np.float64).reshape(-1).copy()
    return best, overlap, score


def all_gather_packed(packed, group=None):
    """All-gather equal-sized [n, 4] int32 result blocks (torch tensor in, torch tensor out),
    rank order = shard order."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    out = torch.empty((world * packed.shape[0], 4), dtype=packed.dtype, device=packed.device)
    dist.all_gather_into_tensor(out, packed.contiguous(), group=group)
    return out


def gather_packed_to0(packed, group=None):
    """Gather equal-sized [n, 4] int32 result blocks to rank 0 (``dist.gather``: RCCL send/recv
    over xGMI with the nccl backend); rank 0 gets the [world * n, 4] tensor in shard order, the
    other ranks None."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    parts = [torch.empty_like(packed) for _ in range(world)] if rank == 0 else None
    dist.gather(packed.contiguous(), gather_list=parts, dst=0, group=group)
    return torch.cat(parts) if rank == 0 else None


class SharedResults:
    """Rank 0's host buffer for the whole job's match results, shared with the node's other ranks
    through POSIX shared memory: [world * F] best (i32) | overlap (u32) | score (f64). Rank r
    writes its shard straight into its slice (its D2H lands there), so after one barrier every
    result is in rank 0's memory with no second copy -- the host form of the gather that
    Dice#matches_by_similarity's per-file results (dice.rb:34-41) need.

    Rank 0 creates the segment (``create=True``) before the others attach by name; rank 0 unlinks
    it in :meth:`close`."""

    def __init__(self, name: str, world: int, files_per_rank: int, create: bool):
        from multiprocessing import shared_memory
        self.world, self.n_per, self.n = world, files_per_rank, world * files_per_rank
        self.create = create
        size = max(16 * self.n, 16)
        if create:
            self.shm = shared_memory.SharedMemory(name=name, create=True, size=size)
        else:
            self.shm = shared_memory.SharedMemory(name=name)
            # the creator owns the segment: keep this process's tracker from unlinking it at exit
            try:
                from multiprocessing import resource_tracker
                resource_tracker.unregister(self.shm._name, 'shared_memory')
            except Exception:
                pass
        buf = self.shm.buf
        self.best = np.ndarray((self.n,), np.int32, buffer=buf, offset=0)
        self.overlap = np.ndarray((self.n,), np.uint32, buffer=buf, offset=4 * self.n)
        self.score = np.ndarray((self.n,), np.float64, buffer=buf, offset=8 * self.n)
        self.nbytes = 16 * self.n

    @property
    def base_ptr(self) -> int:
        return self.best.ctypes.data

    def slice(self, rank: int):
        """Views of rank ``rank``'s [F] region in each array."""
        lo, hi = rank * self.n_per, (rank + 1) * self.n_per
        return self.best[lo:hi], self.overlap[lo:hi], self.score[lo:hi]

    def close(self):
        # drop the numpy views first: SharedMemory.close() refuses while exported buffers live
        self.best = self.overlap = self.score = None
        self.shm.close()
        if self.create:
            self.shm.unlink()


def shm_gather(group_barrier, results: SharedResults, rank: int, write_local) -> None:
    """Host gather: ``write_local(best, overlap, score)`` fills this rank's slice of the shared
    buffer (e.g. a D2H of the rank's device results), then every rank meets at the barrier; on
    return rank 0 holds the whole job's results in ``results``."""
    write_local(*results.slice(rank))
    group_barrier()


class _DeviceArray:
    """``__cuda_array_interface__`` view of a device buffer owned by the C-ABI (no copy)."""

    def __init__(self, ptr: int, n: int, typestr: str):
        self.__cuda_array_interface__ = {'shape': (n,), 'typestr': typestr, 'data': (int(ptr), False),
                                         'version': 2}


def device_results_packed(batch):
    """The resident match results of a ``DeviceBatch`` (``dice_batch_result_ptrs``) packed on
    the device into one int32 [n, 4] torch tensor, ready for the collective -- zero-copy views of
    the library's buffers, one packing copy on the current stream."""
    import torch
    pb, po, ps = batch.result_ptrs()
    n = batch.n
    best = torch.as_tensor(_DeviceArray(pb, n, '<i4'), device='cuda')
    ov = torch.as_tensor(_DeviceArray(po, n, '<i4'), device='cuda')
    score = torch.as_tensor(_DeviceArray(ps, 2 * n, '<i4'), device='cuda').view(n, 2)
    out = torch.empty((n, 4), dtype=torch.int32, device='cuda')
    out[:, 0] = best
    out[:, 1] = ov
    out[:, 2:4] = score
    return out
