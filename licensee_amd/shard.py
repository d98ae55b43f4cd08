"""Multi-GPU sharding of the Dice path (one process per GPU, torch.distributed).

Files are independent and templates are read-only, so each rank scores a
contiguous, disjoint shard with its own replicated template context -- no data-path
collective. Only the 16-byte per-file results move, once, after scoring:

  * ``host``       -- every rank copies its results to host memory (D2H);
  * ``collective`` -- results are packed into one int32 [n, 4] tensor per rank
                      (best, overlap, score as two int32 words) and all-gathered
                      (RCCL over xGMI with the nccl backend, gloo on CPU).

bench.py times both and reports the faster one; tests/test_distributed.py runs the
collective with gloo at world size 2.
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
