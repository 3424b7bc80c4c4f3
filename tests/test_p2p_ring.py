"""The ring algorithms' point-to-point branch (dccl_amd/csrc/algorithms.cpp: the path the RCCL transport and
any plugged-in transport take) at W = 2..8, on the CPU.

tests/native/ring_p2p_harness.cpp links algorithms.cpp with a fake exchange between W thread-ranks that
records every call, and with the oracle as the combine.  Checked here:
  * every exchange of every rank: (to, from, send offset, receive offset, bytes) in order, against the
    reference's step formulas: reduce_scatter_ring.cpp:64-101 (send chunk r-s to r+1, receive chunk r-s-1's
    partial from r-1 into the scratchpad, combine), all_gather_ring.cpp:44-64, all_reduce_ring.cpp:59-72
    (all-gather with new rank r+1), ncclReduceScatter's rank maps (dccl.cpp:626-630) and the recursive
    halving / doubling schedule of all_reduce_recursive_halving_and_doubling.cpp:72-196;
  * every rank's final buffer, bit for bit, against tests/ringsim.py / tests/rabsim.py + the oracle.
The GPU side of the same branch (real combine, the dccl_api glue) is tests/test_p2p_transport.py.
"""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

import oracle
from tests import rabsim, ringsim

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "build", "tests")
HARNESS = os.path.join(OUT, "ring_p2p_harness")
SRCS = [os.path.join(ROOT, "tests", "native", "ring_p2p_harness.cpp"),
        os.path.join(ROOT, "dccl_amd", "csrc", "algorithms.cpp"), os.path.join(ROOT, "oracle", "host_reduce.c"),
        os.path.join(ROOT, "dccl_amd", "csrc", "grouped.cpp")]
SEED = 0xDCC1


@pytest.fixture(scope="module")
def harness():
    deps = SRCS + [os.path.join(ROOT, "dccl_amd", "csrc", f) for f in ("algorithms.hpp", "comm.hpp", "dispatch.hpp",
                                                                        "rccl_transport.hpp")]
    if not os.path.exists(HARNESS) or os.path.getmtime(HARNESS) < max(os.path.getmtime(p) for p in deps):
        # Per-process scratch directory and an atomic rename: pytest-xdist workers may build at once.
        tmp = os.path.join(OUT, f"tmp.{os.getpid()}")
        os.makedirs(tmp, exist_ok=True)
        hip = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-std=c++17", "-O1", "-Wall",
               f"-I{ROOT}/include", f"-I{ROOT}/dccl_amd/csrc"]
        subprocess.run(hip + ["-c", SRCS[0], "-o", f"{tmp}/harness.o"], check=True)
        subprocess.run(hip + ["-c", SRCS[1], "-o", f"{tmp}/algorithms.o"], check=True)
        subprocess.run(hip + ["-c", SRCS[3], "-o", f"{tmp}/grouped.o"], check=True)
        subprocess.run(["gcc", "-std=c11", "-O2", "-fPIC", "-c", SRCS[2], "-o", f"{tmp}/oracle_host_reduce.o"],
                       check=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", f"{tmp}/harness.o", f"{tmp}/algorithms.o",
                        f"{tmp}/grouped.o", f"{tmp}/oracle_host_reduce.o", "-o", f"{tmp}/ring_p2p_harness",
                        "-pthread"], check=True)
        os.replace(f"{tmp}/ring_p2p_harness", HARNESS)
        shutil.rmtree(tmp, ignore_errors=True)
    return HARNESS


def run(harness, tmp_path, algo, W, count, dt, op):
    p = subprocess.run([harness, algo, str(W), str(count), str(dt), str(op), str(tmp_path)], capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    res = json.loads(p.stdout)
    npd = oracle.NP_DTYPES[dt]
    bufs = [np.fromfile(os.path.join(tmp_path, f"rank{r}.bin"), dtype=npd) for r in range(W)]
    return res["rc"], res["log"], bufs


def inputs(W, count, dt, op):
    return [oracle.synth(count, dt, op, SEED, r) for r in range(W)]


def combine_with(dt, op):
    def combine(send, recv):
        assert oracle.expected_reduce(np.ascontiguousarray(send), recv, dt, op) == 0
    return combine


def copy(dst, src):
    dst[:] = src


# ---- the reference's message schedules, as (to, from, send_off, recv_off, send_bytes, recv_bytes); -1 in
# recv_off is the scratchpad, -2 no buffer, -1 in to/from no peer
def ring_log(W, r, slot_bytes, phase, to_new=lambda x: x, to_old=lambda x: x):
    nr = to_new(r)
    to, frm = to_old((nr + 1) % W), to_old((nr - 1) % W)
    out = []
    for s in range(W - 1):
        send = slot_bytes * ((nr - s) % W)
        recv = -1 if phase == "rs" else slot_bytes * ((nr - s - 1) % W)
        out.append([to, frm, send, recv, slot_bytes, slot_bytes])
    return out


def rab_log(W, me, total):
    k = W.bit_length() - 1
    sub, rem = 1 << k, W - (1 << k)
    half = total // 2
    to_new = (lambda o: o // 2 if o < 2 * rem else o - rem)
    to_old = (lambda q: 2 * q if q < rem else q + rem)
    leader, follower = me < 2 * rem and me % 2 == 0, me < 2 * rem and me % 2 == 1
    out = []
    if leader:
        out += [[me + 1, me + 1, half, -1, half, half], [-1, me + 1, -2, half, 0, half]]
    elif follower:
        out += [[me - 1, me - 1, 0, -1, half, half], [me - 1, -1, half, -2, half, 0]]
    if not follower:
        my = to_new(me)
        lo, nbytes = 0, total
        for s in range(k):
            peer = to_old(my ^ (1 << s))
            nbytes //= 2
            keep, give = (lo + nbytes, lo) if (my >> s) & 1 else (lo, lo + nbytes)
            out.append([peer, peer, give, -1, nbytes, nbytes])
            lo = keep
        slice_ = total // sub
        block = int(format(my, f"0{k}b")[::-1], 2) if k else 0
        for s in range(k):
            peer = to_old(my ^ (1 << (k - s - 1)))
            block &= ~((1 << s) - 1)
            ln = slice_ << s
            out.append([peer, peer, block * slice_, (block ^ (1 << s)) * slice_, ln, ln])
    if leader:
        out.append([me + 1, -1, 0, -2, total, 0])
    elif follower:
        out.append([-1, me - 1, -2, 0, 0, total])
    return out


CASES = [(7, 0), (3, 0), (7, 2), (4, 1), (9, 3), (0, 1)]  # (dtype, op): f32 Sum, u32 Sum, f32 Max, i64 Prod, ...


@pytest.mark.parametrize("W", [2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("algo", ["rs", "rs_api", "ag", "ar", "rab"])
def test_p2p_branch_schedule_and_result_cpu(harness, tmp_path, W, algo):
    for dt, op in CASES:
        count = 840 * (1 + (dt % 3))  # divisible by every W <= 8 and by 2^floor(log2 W)
        esz = oracle.NP_DTYPES[dt]().itemsize
        slot_bytes = count // W * esz
        rc, log, got = run(harness, tmp_path, algo, W, count, dt, op)
        assert rc == [0] * W, (algo, W, dt, op, rc)
        want = inputs(W, count, dt, op)
        comb = combine_with(dt, op)
        if algo == "rs":
            ringsim.reduce_scatter_ring(want, comb)
            logs = [ring_log(W, r, slot_bytes, "rs") for r in range(W)]
        elif algo == "rs_api":
            tn, to = ringsim.rs_maps()
            ringsim.reduce_scatter_ring(want, comb, tn, to)
            logs = [ring_log(W, r, slot_bytes, "rs", lambda x: tn(x, W), lambda x: to(x, W)) for r in range(W)]
        elif algo == "ag":
            ringsim.all_gather_ring(want, copy)
            logs = [ring_log(W, r, slot_bytes, "ag") for r in range(W)]
        elif algo == "ar":
            ringsim.ring_allreduce(want, comb, copy)
            logs = [ring_log(W, r, slot_bytes, "rs") +
                    ring_log(W, r, slot_bytes, "ag", lambda x: (x + 1) % W, lambda x: (x - 1) % W) for r in range(W)]
        else:
            rabsim.rabenseifner_allreduce(want, comb)
            logs = [rab_log(W, r, count * esz) for r in range(W)]
        for r in range(W):
            assert log[r] == logs[r], (algo, W, r, log[r][:4], logs[r][:4])
            assert got[r].tobytes() == want[r].tobytes(), (algo, W, dt, op, r)


def grouped_log(W, r, slot_bytes, shift, gather):
    """grouped.cpp's exchanges: to every peer p its part of the slot p owns, then from every peer into the
    scratch (offset -3: inside the scratch), in peer order; then, for the all-reduce, the owned slot to every
    peer and every peer's owned slot into place."""
    peers = [p for p in range(W) if p != r]
    out = [[p, -1, slot_bytes * ((p + shift) % W), -2, slot_bytes, 0] for p in peers]
    out += [[-1, p, -2, -3, 0, slot_bytes] for p in peers]
    if gather:
        out += [[p, -1, slot_bytes * ((r + 1) % W), -2, slot_bytes, 0] for p in peers]
        out += [[-1, p, -2, slot_bytes * ((p + 1) % W), 0, slot_bytes] for p in peers]
    return out


@pytest.mark.parametrize("W", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("algo", ["grs", "grs_api", "gar"])
def test_grouped_schedule_and_result_cpu(harness, tmp_path, W, algo):
    """The grouped RCCL forms (grouped.cpp): every exchange (peer, offset, bytes) and every owned slot (all of the
    all-reduce's buffer) bit-exact against the ring simulation: the chain applies the ring's operations in the
    ring's order."""
    for dt, op in CASES:
        count = 840 * (1 + (dt % 3))
        esz = oracle.NP_DTYPES[dt]().itemsize
        slot = count // W
        rc, log, got = run(harness, tmp_path, algo, W, count, dt, op)
        assert rc == [0] * W, (algo, W, dt, op, rc)
        want = inputs(W, count, dt, op)
        comb = combine_with(dt, op)
        if algo == "gar":
            ringsim.ring_allreduce(want, comb, copy)
        elif algo == "grs":
            ringsim.reduce_scatter_ring(want, comb)
        else:
            tn, to = ringsim.rs_maps()
            ringsim.reduce_scatter_ring(want, comb, tn, to)
        shift = 0 if algo == "grs_api" else 1
        for r in range(W):
            assert log[r] == grouped_log(W, r, slot * esz, shift, algo == "gar"), (algo, W, r, log[r][:4])
            if algo == "gar":
                assert got[r].tobytes() == want[r].tobytes(), (algo, W, dt, op, r)
            else:
                m = (r + shift) % W
                assert got[r][m * slot:(m + 1) * slot].tobytes() == want[r][m * slot:(m + 1) * slot].tobytes(), \
                    (algo, W, dt, op, r)


def test_p2p_branch_rejects_bad_counts_cpu(harness, tmp_path):
    rc, log, _ = run(harness, tmp_path, "rs", 4, 1022, 7, 0)  # count % W != 0 (reduce_scatter_ring.cpp:53-58)
    assert rc == [4] * 4 and log == [[]] * 4
    rc, log, _ = run(harness, tmp_path, "rab", 8, 1020, 7, 0)  # count % 2^k != 0 (:50-54)
    assert rc == [4] * 8 and log == [[]] * 8
