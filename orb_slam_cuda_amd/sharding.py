"""Frame sharding across GPUs (one process per GPU, no data-path collective).

ORB extraction is independent per frame (extractor state is read-only across
calls, src/ORBextractor.cc:496-560) and matching frame t needs only frame
t-1, so frames shard by contiguous blocks per rank; the only cross-rank
dependency is the t-1 frame at a block boundary, which each rank recomputes
(or carries) locally. The control plane (barrier, max-over-ranks of the timed
region) runs over torch.distributed with the gloo backend on the CPU.
"""
from __future__ import annotations

import os


def rank_info() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def shard_frames(n_frames: int, rank: int, world: int) -> range:
    """Contiguous block of a stream of n_frames for `rank` (sizes differ by <= 1)."""
    base, extra = divmod(n_frames, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def boundary_frame(block: range) -> int | None:
    """Index of the frame t-1 a block needs from its predecessor (None for the first)."""
    return block.start - 1 if block.start > 0 else None


def split_sequence(n_frames: int, rank: int, world: int) -> tuple[range, int | None]:
    """ONE sequence of n_frames split over `world` ranks (bench.py
    --split-sequence): the rank's contiguous block and the
    frame t-1 its first pair needs from the block before (None for rank 0).
    One process per GPU holds no other rank's device memory, so the rank
    extracts that boundary frame itself (one extra frame per block) instead of
    receiving its descriptors from rank - 1: no data-path exchange."""
    block = shard_frames(n_frames, rank, world)
    return block, boundary_frame(block)


def sequence_seed(rank: int, base: int = 1000) -> int:
    """Seed of the synthetic sequence a rank streams in the benchmark (one per GPU, C5)."""
    return base + rank


def init_control_plane():
    """gloo process group for barrier / max-reduce; None when world_size == 1."""
    rank, world, _ = rank_info()
    if world <= 1:
        return None
    import torch.distributed as dist
    if not dist.is_initialized():
        dist.init_process_group("gloo")
    return dist


def max_over_ranks(x: float, dist) -> float:
    if dist is None:
        return x
    import torch
    t = torch.tensor([float(x)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: float, dist) -> float:
    if dist is None:
        return x
    import torch
    t = torch.tensor([float(x)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())
