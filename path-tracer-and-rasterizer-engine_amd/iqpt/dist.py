"""Multi-GPU partition of the frame: cyclic pixel rows, one rank per GPU.

Row r of the frame belongs to rank r mod N. A pixel's result depends only on its own XORWOW
stream (keyed by the GLOBAL pixel id, path_tracer.cu:43/338), the packet and the camera, so the
ranks never exchange data while rendering; the only collective is the final gather of the float4
accumulators to rank 0 (RCCL over xGMI on the MI355X node, gloo in the CPU tests), after which
rank 0 de-interleaves the rows.
"""
from __future__ import annotations

import numpy as np

from ._lib import PixelSet


def rows_of(height: int, rank: int, world: int) -> np.ndarray:
    return np.arange(rank, height, world)


def max_rows(height: int, world: int) -> int:
    return (height + world - 1) // world


def pixel_set_for_rank(width: int, height: int, rank: int, world: int) -> PixelSet:
    n = len(rows_of(height, rank, world))
    return PixelSet(0, width, rank, world, n)


def assemble(parts, width: int, height: int, world: int, channels: int = 4):
    """parts[r]: rank r's compact rows (padded to max_rows*width pixels). Works on numpy or torch."""
    first = parts[0]
    if hasattr(first, "new_empty"):
        full = first.new_empty((height, width, channels))
    else:
        full = np.empty((height, width, channels), dtype=first.dtype)
    for r in range(world):
        rows = rows_of(height, r, world)
        blk = parts[r].reshape(-1, width, channels)[: len(rows)]
        if hasattr(full, "new_empty"):
            import torch
            full[torch.as_tensor(rows, device=full.device)] = blk
        else:
            full[rows] = blk
    return full.reshape(height * width, channels)
