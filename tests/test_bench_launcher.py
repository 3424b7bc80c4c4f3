"""bench.py's launcher on the CPU: `--gpus N` without WORLD_SIZE starts N rank processes itself (one per GPU,
as the reference's harness runs one process per rank, /root/reference/README.md:74-101), and a `--gpus`
that disagrees with a launcher's WORLD_SIZE is an error.  The GPU rehearsal of the same launcher is
tests/test_bench_gpu.py::test_bench_self_launch_two_ranks_one_gpu."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, "bench.py", *args], cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=timeout)


def test_gpus_must_match_world_size():
    p = _run(["--gpus", "1"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert p.returncode == 2 and "WORLD_SIZE=2" in p.stderr, p.stderr
    p = _run(["--gpus", "4"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert p.returncode == 2 and "--gpus 4" in p.stderr, p.stderr


def test_self_launch_needs_the_gpus():
    import torch
    if torch.cuda.device_count() >= 2:
        return
    p = _run(["--gpus", "2"])
    assert p.returncode == 2 and "needs 2 GPUs" in p.stderr, p.stderr


def test_self_launch_starts_n_ranks():
    for n in (2, 3):
        p = _run(["--gpus", str(n), "--launcher-selftest"], {"DCCL_BENCH_BACKEND": "gloo"})
        assert p.returncode == 0, p.stderr[-2000:]
        lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        assert len(lines) == 1, p.stdout
        res = json.loads(lines[0])
        assert res["n_gpus"] == n and res["rank_sum"] == n * (n - 1) // 2, res
        assert res["local_rank"] == "0" and res["master"].startswith("127.0.0.1:"), res


def test_rccl_rehearsal_gives_each_rank_a_host_id():
    """DCCL_BENCH_RCCL_REHEARSAL=1: N RCCL ranks on fewer GPUs, each rank with its own NCCL_HOSTID (RCCL joins them
    over loopback sockets instead of refusing two ranks on one device); without it, an RCCL run on too few GPUs is
    refused (test_self_launch_needs_the_gpus)."""
    p = _run(["--gpus", "3", "--launcher-selftest"], {"DCCL_BENCH_BACKEND": "nccl", "DCCL_BENCH_RCCL_REHEARSAL": "1"})
    assert p.returncode == 0, p.stderr[-2000:]
    res = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    ids = res["nccl_hostids"]
    assert res["n_gpus"] == 3 and len(set(ids)) == 3 and all(i.startswith("dccl-rehearsal-") for i in ids), res
    p = _run(["--gpus", "2", "--launcher-selftest"], {"DCCL_BENCH_BACKEND": "gloo"})
    assert json.loads(p.stdout.strip().splitlines()[-1])["nccl_hostids"] == [None, None]


def test_self_launch_fails_when_a_rank_fails():
    p = _run(["--gpus", "2", "--launcher-selftest"], {"DCCL_BENCH_BACKEND": "gloo",
                                                       "DCCL_BENCH_SELFTEST_FAIL_RANK": "1"})
    assert p.returncode == 7, (p.returncode, p.stderr[-2000:])
    assert "rank exit codes [0, 7]" in p.stderr


def test_name_tables_match_the_package():
    import bench
    import dccl_amd
    assert bench.DTYPE_NAMES == dccl_amd.DTYPE_NAMES
    assert bench.OP_NAMES == {k: v for k, v in dccl_amd.OP_NAMES.items() if k != "avg"}
    assert bench.dccl_amd is None  # importing bench loads no native library


def test_allreduce_summary_keeps_the_flags():
    import bench
    ar = {"count": 8, "ring": {"int32_sum_bit_exact_vs_rccl": True, "fp32_within_bound": True, "ms": 1.0,
                               "busbw_gb_s": 2.0, "fp32_max_abs_diff_vs_rccl": 0.0},
          "rccl_allreduce": {"ms": 1.5, "busbw_gb_s": 1.0, "backend": "nccl"},
          "fp32_direct_bit_exact_vs_ring": True, "sweep_busbw_gb_s": {"1": {"ring": 1.0, "rccl": 2.0}},
          "dccl_allgather": {"bytes_per_rank": 4, "direct": {"bit_exact": True, "ms": 0.1, "ms_each": [0.1],
                                                              "busbw_gb_s": 3.0}}}
    s = bench.allreduce_summary(ar)
    assert s["ring"] == {"int32_sum_bit_exact_vs_rccl": True, "fp32_within_bound": True, "ms": 1.0, "busbw_gb_s": 2.0}
    assert s["rccl"] == {"ms": 1.5, "busbw_gb_s": 1.0} and s["fp32_direct_bit_exact_vs_ring"]
    assert s["dccl_allgather"] == {"direct": {"bit_exact": True, "ms": 0.1, "busbw_gb_s": 3.0}}
    assert s["sweep_busbw_gb_s"] == {"1": {"ring": 1.0, "rccl": 2.0}}
    assert bench.allreduce_summary({"error": "x"}) == {"error": "x"}


def test_socket_rehearsal_sizes_only_when_ranks_share_gpus(monkeypatch):
    """The N > 1 child's collectives are sized down only for a socket rehearsal (DCCL_BENCH_RCCL_REHEARSAL=1 with
    more RCCL ranks than GPUs); a real one-GPU-per-rank run keeps 256 MiB all-reduces and C5's full size."""
    import bench
    import torch
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    monkeypatch.setenv("DCCL_BENCH_RCCL_REHEARSAL", "1")
    assert bench.socket_rehearsal(8, "nccl") and not bench.socket_rehearsal(1, "nccl")
    assert not bench.socket_rehearsal(8, "gloo")
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    assert not bench.socket_rehearsal(8, "nccl")
    monkeypatch.delenv("DCCL_BENCH_RCCL_REHEARSAL")
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    assert not bench.socket_rehearsal(8, "nccl")
    assert bench.REHEARSAL_CHILD_TIMEOUT_S > bench.CHILD_TIMEOUT_S and bench.REHEARSAL_AR_MIB < 256
