"""Multi-rank host logic on CPU (gloo, world_size 2 and 3): the contiguous shard partition and the
all-gather that hands every rank the full combined buffer (the one exchange step of BASELINE
config C5).  The per-shard combine here is the oracle (test infrastructure); on the GPU box the
same partition drives the HIP kernel (bench.py --total-gib)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from dccl_amd.shard import all_bounds, shard_bounds


def test_partition_covers_exactly_once():
    for count in [0, 1, 63, 64, 65, 1000, 4099, 1 << 20, (1 << 20) + 7]:
        for esz in (1, 2, 4, 8):
            for world in (1, 2, 3, 4, 7, 8):
                b = all_bounds(count, esz, world)
                assert b[0][0] == 0 and b[-1][1] == count
                for (s0, e0), (s1, e1) in zip(b, b[1:]):
                    assert e0 == s1 and s0 <= e0
                for s, _ in b[:-1] + [b[-1]]:
                    assert (s * esz) % 256 == 0
    with pytest.raises(ValueError):
        shard_bounds(10, 4, 2, 2)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, count, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(42)  # every rank builds the same global operands
    send = rng.standard_normal(count).astype(np.float32)
    recv = rng.standard_normal(count).astype(np.float32)
    s, e = shard_bounds(count, 4, world, rank)
    mine = oracle.combine(send[s:e], recv[s:e], 7, 0)
    bounds = all_bounds(count, 4, world)
    width = max(b - a for a, b in bounds)
    padded = torch.zeros(width, dtype=torch.float32)
    padded[: e - s] = torch.from_numpy(mine)
    out = [torch.zeros(width, dtype=torch.float32) for _ in range(world)]
    dist.all_gather(out, padded)
    full = np.concatenate([out[r][: b - a].numpy() for r, (a, b) in enumerate(bounds)])
    want = oracle.combine(send, recv, 7, 0)
    q.put((rank, full.tobytes() == want.tobytes()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,count", [(2, 100003), (3, 4099)])
def test_sharded_combine_allgather_gloo(world, count):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, count, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    assert all(ok for _, ok in res), res
