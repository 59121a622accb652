"""Multi-GPU partition logic on CPU: world_size-2 gloo processes each unmask
their shard with the oracle; the gathered result equals the single-process
batch, and the harness reductions (max time, byte totals) are right."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from kuma_amd import shard
from oracle import oracle as orc


def test_uniform_ranges_cover():
    for n in (0, 1, 7, 1 << 20, 10485760):
        for world in (1, 2, 3, 8):
            rs = [shard.uniform_range(n, g, world) for g in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in rs]
            assert max(sizes) - min(sizes) <= 1


def test_sub_batches_cover_and_pair_up():
    # BASELINE configs[4]: 10 M frames over 1/2/4/8 GPUs, 80 GiB resident batches
    for job, mb in ((10485760, 1310720), (1 << 20, 1310720), (1 << 20, 262144), (7, 2), (0, 5), (13, 100)):
        for world in (1, 2, 3, 4, 8):
            counts = set()
            for g in range(world):
                n, bs = shard.sub_batches(job, g, world, mb)
                lo, hi = shard.uniform_range(job, g, world)
                counts.add(len(bs))
                assert n <= max(mb, 1)
                assert bs[0][0] == lo and bs[-1][1] == hi
                assert all(b[1] == c[0] for b, c in zip(bs, bs[1:]))
                assert all(0 <= b - a <= n for a, b in bs)
            assert len(counts) == 1  # same sub-batch count on every rank
    n, bs = shard.sub_batches(10485760, 0, 1, 1310720)
    assert n == 1310720 and len(bs) == 8
    assert shard.sub_batches(10485760, 7, 8, 1310720) == (1310720, [(9175040, 10485760)])


def test_byte_balanced_ranges():
    rng = np.random.default_rng(0)
    lens = 128 * 2 ** rng.integers(0, 14, size=5000)
    for world in (1, 2, 4, 8):
        rs = shard.byte_balanced_ranges(lens, world)
        assert rs[0][0] == 0 and rs[-1][1] == len(lens)
        assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
        per = [int(lens[a:b].sum()) for a, b in rs]
        assert max(per) - min(per) <= 2 * int(lens.max())
    assert shard.byte_balanced_ranges([], 4) == [(0, 0)] * 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, L, seed, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    lo, hi = shard.uniform_range(n, rank, world)
    base = orc.synthetic(seed, lo * L, (hi - lo) * L)
    d = np.zeros(hi - lo, dtype=orc.DESC_DTYPE)
    d["off"] = np.arange(hi - lo, dtype=np.uint64) * L
    d["len"] = L
    keys = np.array([orc.splitmix64((seed ^ 0x5EED) + i) & 0xFFFFFFFF for i in range(lo, hi)], dtype=np.uint32)
    d["key"] = keys
    orc.unmask_batch(base, d)
    # per-rank checksum (sum of 64-bit words, wrapping) + byte count; elapsed stand-in = rank + 1
    cs = int(base.view(np.uint64).sum(dtype=np.uint64)) if len(base) else 0
    t = torch.tensor([cs & 0xFFFFFFFF, (hi - lo) * L], dtype=torch.int64)
    dist.all_reduce(t)  # sum over ranks
    el = torch.tensor([float(rank + 1)])
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    if rank == 0:
        out.put((int(t[0]), int(t[1]), float(el[0])))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_unmask_matches_single_process(world):
    n, L, seed = 64, 4096, 77
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, L, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    cs_sum, nbytes, el = q.get(timeout=10)
    # single process reference
    base = orc.synthetic(seed, 0, n * L)
    d = np.zeros(n, dtype=orc.DESC_DTYPE)
    d["off"] = np.arange(n, dtype=np.uint64) * L
    d["len"] = L
    d["key"] = np.array([orc.splitmix64((seed ^ 0x5EED) + i) & 0xFFFFFFFF for i in range(n)], dtype=np.uint32)
    orc.unmask_batch(base, d)
    per_rank = []
    for g in range(world):
        lo, hi = shard.uniform_range(n, g, world)
        per_rank.append(int(base[lo * L:hi * L].view(np.uint64).sum(dtype=np.uint64)) & 0xFFFFFFFF)
    assert cs_sum == sum(per_rank)
    assert nbytes == n * L
    assert el == float(world)
    assert shard.aggregate_rate([nbytes // world] * world, [1.0, float(world)]) == nbytes / world
