"""The IPC transport's importer cache (dccl_amd/csrc/ipc_cache.hpp) on the CPU, against a fake runtime that
behaves like ROCm 7.2's dmabuf IPC did in round 3 ("What's weak" #1): opening handle bytes that
are already open returns that import uncounted, and a second close of a base is an error.  The driver
(tests/native/ipc_cache_test.cpp) is built with g++ under ASan + UBSan; it covers the repeated-handle
eviction, the in-use alias refusal, an open that returns a base another key holds, retirement (also while
in use and by log overflow), trimming, size mismatches, open retries and a 500-round churn."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_ipc_cache_against_fake_runtime(tmp_path):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    exe = tmp_path / "ipc_cache_test"
    build = subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-Wall", "-Wextra", "-Werror",
                            "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                            f"-I{os.path.join(ROOT, 'dccl_amd', 'csrc')}",
                            os.path.join(ROOT, "tests", "native", "ipc_cache_test.cpp"), "-o", str(exe)],
                           capture_output=True, text=True, timeout=300)
    assert build.returncode == 0, build.stderr[-3000:]
    run = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert run.returncode == 0, run.stdout + run.stderr[-3000:]
    assert "ipc_cache: ok" in run.stdout
