"""bench.py's multi-GPU-only helpers exercised at world size 1 on the GPU box (the driver runs the
real N = 2/4/8 bench on an 8-GPU node; these keep that code path from being untested)."""
import os
import socket

import pytest

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_dccl_allreduce_rccl_world1():
    import torch
    import torch.distributed as dist

    import bench
    import dccl_amd
    if not dccl_amd.lib.dccl_rccl_available():
        pytest.skip("librccl not loadable")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1, device_id=dev)
    try:
        res, finished = bench.run_with_watchdog(lambda: bench.dccl_allreduce_rccl(1, 0, dev, 1 << 20, iters=2), 120)
        assert finished, res
        assert "error" not in res, res
        assert res["int32_sum_bit_exact_vs_rccl"] and res["fp32_within_bound"]
    finally:
        dist.destroy_process_group()


def test_watchdog_reports_timeout():
    import time

    import bench
    res, finished = bench.run_with_watchdog(lambda: time.sleep(5), 0.2)
    assert not finished and "timed out" in res["error"]
