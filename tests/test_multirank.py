"""world_size-2 gloo tests of the sharding / control-plane path used by bench.py (CPU)."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from orb_slam_cuda_amd import sharding
    from orb_slam_cuda_amd.synth import SynthSequence
    dist = sharding.init_control_plane()
    r, w, lr = sharding.rank_info()
    mx = sharding.max_over_ranks(1.5 + r, dist)
    sm = sharding.sum_over_ranks(10 * (r + 1), dist)
    block = sharding.shard_frames(129, r, w)
    fr = SynthSequence(sharding.sequence_seed(r), 320, 200).frames(2)
    dist.barrier()
    dist.destroy_process_group()
    q.put((r, mx, sm, (block.start, block.stop), sharding.boundary_frame(block), int(fr.sum())))


def test_two_rank_gloo_control_plane():
    pytest.importorskip("torch")
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, mx0, sm0, b0, bf0, s0), (r1, mx1, sm1, b1, bf1, s1) = res
    assert mx0 == mx1 == 2.5          # max of per-rank wall times
    assert sm0 == sm1 == 30.0
    assert b0 == (0, 65) and b1 == (65, 129)  # contiguous, disjoint, covering
    assert bf0 is None and bf1 == 64
    assert s0 != s1                   # each rank streams its own sequence


def test_shard_frames_partition():
    from orb_slam_cuda_amd.sharding import shard_frames
    for n in (0, 1, 7, 64, 1000):
        for w in (1, 2, 3, 8):
            blocks = [shard_frames(n, r, w) for r in range(w)]
            cat = np.concatenate([np.arange(b.start, b.stop) for b in blocks])
            assert np.array_equal(cat, np.arange(n))
            sizes = [len(b) for b in blocks]
            assert max(sizes) - min(sizes) <= 1


def _split_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import hashlib
    from orb_slam_cuda_amd import sharding
    from orb_slam_cuda_amd.synth import SynthStream
    dist = sharding.init_control_plane()
    r, w, _ = sharding.rank_info()
    block, prev = sharding.split_sequence(12, r, w)  # bench.py --split-sequence: pool x world frames
    s = SynthStream(sharding.sequence_seed(0), 160, 120)
    h = lambda a: hashlib.sha1(np.ascontiguousarray(a).tobytes()).hexdigest()
    mine = [h(f) for f in s.frames(block)]
    halo = h(s.frame(prev)) if prev is not None else None
    everyone = [None] * w
    dist.all_gather_object(everyone, (r, block.start, block.stop, prev, mine, halo))
    dist.barrier()
    dist.destroy_process_group()
    q.put(everyone)


def test_split_sequence_blocks_and_boundary_frames():
    """--split-sequence bookkeeping with world_size 2 on gloo: the ranks' blocks
    tile ONE sequence, and the boundary frame rank 1 renders for its first pair
    is byte-identical to the last frame of rank 0's block (frames from
    SynthStream are random-access and rank-independent)."""
    pytest.importorskip("torch")
    import multiprocessing as mp
    from orb_slam_cuda_amd.synth import SynthStream
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_split_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1]
    (r0, a0, b0, p0, m0, h0), (r1, a1, b1, p1, m1, h1) = res[0]
    assert (a0, b0, p0) == (0, 6, None) and (a1, b1, p1) == (6, 12, 5)
    assert h0 is None and h1 == m0[-1]
    assert len(set(m0 + m1)) == 12
    # the stream is the same sequence whoever renders it, in any order
    s = SynthStream(1000, 160, 120)
    later_first = s.frames([7, 2])
    fresh = SynthStream(1000, 160, 120)
    assert np.array_equal(later_first[1], fresh.frame(2)) and np.array_equal(later_first[0], fresh.frame(7))
