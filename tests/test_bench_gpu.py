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


def test_dccl_allreduce_world1(monkeypatch):
    import torch
    import torch.distributed as dist

    import bench
    import dccl_amd
    if not dccl_amd.lib.dccl_rccl_available():
        pytest.skip("librccl not loadable")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    port = _port()
    monkeypatch.setenv("DCCL_BOOTSTRAP_TAG", f"bench_test_{port}")
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    try:
        res, finished = bench.run_with_watchdog(lambda: bench.dccl_allreduce_multi(1, 0, dev, 1 << 20, iters=2), 120)
        assert finished, res
        assert "error" not in res, res
        for name in ("ring", "direct"):
            assert res[name]["int32_sum_bit_exact_vs_rccl"] and res[name]["fp32_within_bound"], res
            assert res[name]["broadcast_bit_exact"] and res[name]["reduce_bit_exact"], res
        assert res["fp32_direct_bit_exact_vs_ring"], res
    finally:
        dist.destroy_process_group()


def test_watchdog_reports_timeout():
    import time

    import bench
    res, finished = bench.run_with_watchdog(lambda: time.sleep(5), 0.2)
    assert not finished and "timed out" in res["error"]


def test_bench_direct_allreduce_two_processes_one_gpu():
    """bench.py's N>1 path rehearsed with two ranks on the box's one GPU: gloo for torch.distributed,
    the direct IPC all-reduce between the two processes checked against gloo's all_reduce."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {**os.environ, "DCCL_BENCH_BACKEND": "gloo", "DCCL_BENCH_AR_TRANSPORTS": "direct",
           "DCCL_BOOTSTRAP_TAG": f"bench_rehearsal_{_port()}"}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2", "--steps", "3",
           "--warmup", "1", "--mib", "64", "--c5-gib", "0.25", "--no-cpu", "--no-host-staged"]
    p = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, p.stdout[-3000:]
    res = json.loads(lines[0])
    c5 = res["c5"]
    assert c5["combine_ms"] > 0 and c5["allgather"]["ms"] > 0, c5
    ar = res["dccl_allreduce"]
    assert "error" not in ar, ar
    assert ar["direct"]["int32_sum_bit_exact_vs_rccl"] and ar["direct"]["fp32_within_bound"], ar
    assert ar["direct"]["broadcast_bit_exact"] and ar["direct"]["reduce_bit_exact"], ar
    assert ar["dccl_allgather"]["direct"]["bit_exact"], ar["dccl_allgather"]
    assert ar["c5_allgather"]["direct"]["bit_exact"], ar["c5_allgather"]


def test_bench_self_launch_two_ranks_one_gpu():
    """Plain `python3 bench.py --gpus 2` (no launcher): bench.py starts its two rank processes itself, here both on
    the box's one GPU (gloo for torch.distributed, the direct IPC collectives between the two processes), and
    prints one line with n_gpus == 2 and its sampled results verified."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update({"DCCL_BENCH_BACKEND": "gloo", "DCCL_BENCH_AR_TRANSPORTS": "direct",
                "DCCL_BOOTSTRAP_TAG": f"bench_self_launch_{_port()}"})
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1", "--mib", "64",
           "--c5-gib", "0.25", "--no-cpu", "--other-pairs", "2"]
    p = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, p.stdout[-3000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["verified"] is True, res
    assert res["c5"]["verified"] and res["other_layout"]["pairs"] == 2, res
    s = res["dccl_allreduce_summary"]
    assert s["direct"]["int32_sum_bit_exact_vs_rccl"] and s["dccl_allgather"]["direct"]["bit_exact"], s
    assert s["direct"]["broadcast_bit_exact"] and s["direct"]["reduce_bit_exact"], s
    assert list(res)[-1] == "verified"


def test_bench_rccl_two_ranks_one_gpu():
    """The driver's default N>1 path (torch.distributed on RCCL, the RCCL all-gather of the shards and of C5, the
    namespace-dccl all_reduce / all_gather / broadcast / reduce over the RCCL p2p ring, RCCL's own all_reduce as
    the check) rehearsed with plain `python3 bench.py --gpus 2` on the box's one GPU: each rank gets its own
    NCCL_HOSTID, so RCCL joins the two ranks over its socket transport on loopback instead of refusing a second
    rank on one device.  rccl_exchange (dccl_amd/csrc/rccl_transport.cpp) runs with two real RCCL ranks."""
    import json
    import subprocess
    import sys
    import dccl_amd
    if not dccl_amd.lib.dccl_rccl_available():
        pytest.skip("librccl not loadable")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update({"DCCL_BENCH_BACKEND": "nccl", "DCCL_BENCH_RCCL_REHEARSAL": "1",
                "DCCL_BOOTSTRAP_TAG": f"bench_rccl_rehearsal_{_port()}"})
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1", "--mib", "64",
           "--c5-gib", "0.25", "--no-cpu", "--other-pairs", "2", "--rank-timeout", "240"]
    p = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, p.stdout[-3000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["verified"] is True and "rehearsal" in res, res
    assert res["allgather"]["ms"] > 0 and res["c5"]["verified"] and res["c5"]["allgather"]["ms"] > 0, res
    s = res["dccl_allreduce_summary"]
    assert "error" not in s, s
    for name in ("ring", "direct"):
        assert s[name]["int32_sum_bit_exact_vs_rccl"] and s[name]["fp32_within_bound"], s
        assert s[name]["broadcast_bit_exact"] and s[name]["reduce_bit_exact"], s
        assert s["dccl_allgather"][name]["bit_exact"], s
    assert s["fp32_direct_bit_exact_vs_ring"] and s["rccl"]["ms"] > 0, s
    assert s["c5_allgather"]["direct"]["bit_exact"], s
    # the grouped RCCL all-reduce and the IPC transport's counters
    assert s["fp32_grouped_bit_exact_vs_ring"] and s["grouped"]["int32_sum_bit_exact_vs_rccl"], s
    assert s["ipc_stats"]["alias_errors"] == 0 and s["ipc_stats"]["scratch_copies"] > 0, s
    # the per-size all-reduce sweep (socket rehearsal: 1 and 4 MiB), every algorithm and RCCL's own
    assert set(s["sweep_busbw_gb_s"]) == {"1", "4"}, s
    assert all(set(r) == {"ring", "grouped", "direct", "rccl"} and min(r.values()) > 0
               for r in s["sweep_busbw_gb_s"].values()), s
    assert s["dccl_allgather"]["direct"]["wrong_slices_all_ranks"] == 0, s
    # the child's wall time per phase, against its watchdog
    assert s["child_wall_s"] < s["child_timeout_s"], s
    assert {"init", "allreduce_ring", "allreduce_grouped", "allreduce_direct", "sweep", "allgather",
            "finalize"} <= set(s["phase_s"]), s["phase_s"]


def test_host_crossover_leg(monkeypatch):
    """bench.py's host_crossover leg, on small sizes: every kind of host operand (registered,
    pinned, pageable) and every leg timed on the same buffers, the GPU results bit-exact against the oracle, the
    crossover keys present, the registration undone."""
    import bench
    import dccl_amd
    bench._native()
    monkeypatch.setattr(bench, "HOST_SIZES", [4 << 10, 1 << 20, 16 << 20])
    monkeypatch.setattr(bench, "HOST_ROTATE_BYTES", 64 << 20)
    res = bench.host_crossover(min_s=0.03)
    assert res["all_bit_exact"] is True, res
    assert [r["bytes"] for r in res["rows"]] == [4 << 10, 1 << 20, 16 << 20]
    for row in res["rows"]:
        for kind in ("registered", "pinned", "pageable"):
            rec = row[kind]
            assert rec["gpu_us"] > 0 and rec["cpu1_us"] > 0 and rec["cpu_all_us"] > 0, rec
    assert set(res["crossover"]) == {"registered", "pinned", "pageable"}
    assert res["product_default_gpu_min_bytes"] == dccl_amd.host_reduce_gpu_min_bytes(7) > 0
    assert dccl_amd.host_reduce_gpu_min_bytes(9) == 0 and dccl_amd.host_reduce_gpu_min_bytes(6) == 0


def test_bench_single_gpu_line():
    """bench.py at N=1 prints exactly one JSON line with the contract's keys, the C5 extra and the C3 / C4
    legs (every C3 entry sample-verified)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--mib", "64", "--c5-gib", "0.5",
           "--no-host-staged", "--cpu-seconds", "1"]
    p = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout[-3000:]
    res = json.loads(lines[0])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert key in res, key
    assert res["n_gpus"] == 1 and res["value"] > 0
    assert res["roofline"]["bound"] == "hbm" and 0 < res["roofline"]["frac"] < 1.5
    assert res["cpu_baseline"]["cores"] >= 1 and res["cpu_baseline"]["value"] > 0
    c5 = res["c5"]
    assert c5["scaling"] == "strong" and c5["combine_ms"] > 0 and "allgather" not in c5
    assert len(res["c3"]) == 20 and all(r["verified"] for r in res["c3"]), res["c3"]
    sizes = [r["bytes_per_operand"] for r in res["c4"]]
    assert sizes == [1 << e for e in range(12, 33)] and all(r["us_per_launch"] > 0 for r in res["c4"])
    assert all(r["graph_us_per_launch"] > 0 for r in res["c4"] if r["bytes_per_operand"] <= 64 << 20)
    assert all(r["native_eager_us_per_launch"] > 0 for r in res["c4"] if r["bytes_per_operand"] <= 64 << 20)
    assert res["other_layout"]["layout"] == "separate" and res["other_layout"]["pairs"] == 4
    assert res["verified"] is True and list(res)[-1] == "verified"
    cb = res["cpu_baseline"]
    q = cb["cgroup_cpu_quota"]
    granted = max(1, min(cb["affinity_cpus"], int(q))) if q else cb["affinity_cpus"]
    assert cb["all_cores"]["cores"] == granted  # the quota's CPUs, not a throttled thread per affinity CPU
    assert (cb["affinity_threads"] is None) == (cb["affinity_cpus"] <= granted)
