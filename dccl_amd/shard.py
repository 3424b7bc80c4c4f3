"""Contiguous sharding of one buffer across the GPUs of a node.

The combine is element-wise, so a buffer of `count` elements splits into G contiguous slices,
one per GPU, with no communication for the combine itself.  Slice starts are aligned to
`align_bytes` (default 256 B: whole 128-B lines and 16-B vectors for every dtype); the last
slice takes the remainder.  This mirrors the reference's own slot partition
(`count/W` contiguous elements, /root/reference/src/core/reduce_scatter_ring.cpp:22,64-65)
without its `count % W == 0` restriction.
"""
from __future__ import annotations


def shard_bounds(count: int, elem_size: int, world: int, rank: int, align_bytes: int = 256) -> tuple[int, int]:
    """Element range [start, stop) owned by `rank`."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    if align_bytes % elem_size:
        raise ValueError("alignment must be a multiple of the element size")
    unit = align_bytes // elem_size
    units = count // unit
    per = units // world
    extra = units % world
    start_u = rank * per + min(rank, extra)
    stop_u = start_u + per + (1 if rank < extra else 0)
    start = start_u * unit
    stop = count if rank == world - 1 else stop_u * unit
    return start, stop


def all_bounds(count: int, elem_size: int, world: int, align_bytes: int = 256) -> list[tuple[int, int]]:
    return [shard_bounds(count, elem_size, world, r, align_bytes) for r in range(world)]
