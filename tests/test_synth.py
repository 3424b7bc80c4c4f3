"""Counter-based synthetic operands (include/dccl/dccl_synth.h) and the full-size
parity they enable.

CPU: the oracle's C generator against the published splitmix64 known answer and an independent
numpy restatement of the value mapping; the C-ABI's argument checks.
GPU: the device generator bit-exact against the oracle's, and BASELINE config C3 at its full size
(1 GiB per operand x {fp16, bf16, fp32, int32, int64} x Sum/Prod/Max/Min, plus the Avg error):
operands generated on the device, combined by the HIP kernel, and compared bit for bit with the
oracle combine of the host-regenerated operands.
"""
import numpy as np
import pytest

import oracle

SEED = 0xDCC1
M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def np_splitmix64(z: np.ndarray) -> np.ndarray:
    z = z + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def np_synth(n, dt, op, seed, buffer_id, first=0):
    """Independent numpy restatement of the value mapping in include/dccl/dccl_synth.h."""
    key = np.uint64(seed) ^ (np.uint64(buffer_id) << np.uint64(40))
    x = np_splitmix64(key ^ np.arange(first, first + n, dtype=np.uint64))
    top = x >> np.uint64(63)
    if dt in (0, 1, 2, 3, 4, 5):
        return x.astype(oracle.NP_DTYPES[dt])  # numpy truncates to the low bytes
    if op == 1:  # [0.5, 2): exponent 2^-1 / 2^0, random mantissa
        if dt == 7:
            return (((np.uint64(126) + top) << np.uint64(23)) | (x & np.uint64(0x7FFFFF))).astype(np.uint32).view(np.float32)
        if dt == 8:
            return (((np.uint64(1022) + top) << np.uint64(52)) | (x & np.uint64((1 << 52) - 1))).view(np.float64)
        if dt == 6:
            return (((np.uint64(14) + top) << np.uint64(10)) | (x & np.uint64(0x3FF))).astype(np.uint16)
        return (((np.uint64(126) + top) << np.uint64(7)) | (x & np.uint64(0x7F))).astype(np.uint16)
    if dt == 7:
        return ((x >> np.uint64(40)).astype(np.int64) - (1 << 23)).astype(np.float32) * np.float32(2.0 ** -23)
    if dt == 8:
        return ((x >> np.uint64(11)).astype(np.int64) - (1 << 52)).astype(np.float64) * 2.0 ** -52
    if dt == 6:
        v = ((x >> np.uint64(53)).astype(np.int64) - (1 << 10)).astype(np.float64) * 2.0 ** -10
        return v.astype(np.float16).view(np.uint16)  # exact: no rounding
    v = ((x >> np.uint64(56)).astype(np.int64) - (1 << 7)).astype(np.float32) * np.float32(2.0 ** -7)
    return (v.view(np.uint32) >> np.uint32(16)).astype(np.uint16)  # exact: low 16 bits are zero


def test_splitmix64_known_answer_cpu():
    # splitmix64 with state 0: first output 0xe220a8397b1dcdaf (published test vector)
    assert int(oracle.synth(1, 5, 0, 0, 0)[0]) == 0xE220A8397B1DCDAF
    assert int(np_splitmix64(np.zeros(1, np.uint64))[0]) == 0xE220A8397B1DCDAF


@pytest.mark.parametrize("dt", list(range(10)))
@pytest.mark.parametrize("op", [0, 1])
def test_oracle_synth_matches_numpy_restatement_cpu(dt, op):
    for first in (0, 12345):
        a = oracle.synth(4099, dt, op, SEED, 1, first)
        b = np_synth(4099, dt, op, SEED, 1, first)
        assert a.tobytes() == b.tobytes(), (dt, op, first)


@pytest.mark.parametrize("dt", [6, 7, 8, 9])
def test_synth_value_ranges_cpu(dt):
    n = 1 << 16
    to_f = {6: lambda a: a.view(np.float16).astype(np.float64), 9: lambda a: (a.astype(np.uint32) << 16).view(np.float32).astype(np.float64),
            7: lambda a: a.astype(np.float64), 8: lambda a: a}[dt]
    s = to_f(oracle.synth(n, dt, 0, SEED, 0))
    p = to_f(oracle.synth(n, dt, 1, SEED, 0))
    assert s.min() >= -1 and s.max() < 1 and abs(s.mean()) < 0.05
    assert p.min() >= 0.5 and p.max() < 2
    assert np.isfinite(s).all() and np.isfinite(p).all()


def test_synth_fill_argument_checks_cpu():
    import dccl_amd
    assert dccl_amd.synth_fill(0, 10, 16, 0, SEED, 0) == 4   # bad dtype
    assert dccl_amd.synth_fill(0, -1, 16, 0, SEED, 0) == 4
    assert dccl_amd.synth_fill(0, 7, 16, 7, SEED, 0) == 4    # bad op
    assert dccl_amd.synth_fill(0, 7, 16, 0, SEED, 0) == 4    # NULL with count > 0
    assert dccl_amd.synth_fill(0, 7, 0, 0, SEED, 0) == 0     # count 0: nothing to do


# ----------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("dt", list(range(10)))
@pytest.mark.parametrize("op", [0, 1])
def test_device_synth_matches_oracle(gpu, dt, op):
    import torch
    import dccl_amd
    esz = dccl_amd.size_of_type(dt)
    for n, off in ((1, 0), (17, 0), (4099, 2 * esz), ((1 << 20) + 5, 8), ((1 << 20) + 5, 0)):
        t = torch.full((n * esz + off + 64,), 0xA5, dtype=torch.uint8, device="cuda")
        assert dccl_amd.synth_fill(t.data_ptr() + off, dt, n, op, SEED, 3) == 0
        torch.cuda.synchronize()
        h = t.cpu().numpy()
        assert h[off:off + n * esz].tobytes() == oracle.synth(n, dt, op, SEED, 3).tobytes(), (n, off)
        assert (h[:off] == 0xA5).all() and (h[off + n * esz:] == 0xA5).all()  # nothing outside


C3 = [(6, "fp16"), (9, "bf16"), (7, "fp32"), (2, "int32"), (4, "int64")]


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.parametrize("dt,name", C3)
def test_c3_full_size_against_oracle(gpu, dt, name):
    """BASELINE config C3 at its full size: 1 GiB per operand, every op, bit-exact vs the oracle."""
    import torch
    import dccl_amd
    esz = dccl_amd.size_of_type(dt)
    n = (1 << 30) // esz
    send = torch.empty(n * esz, dtype=torch.uint8, device="cuda")
    recv = torch.empty_like(send)
    for op in (0, 1, 2, 3):
        assert dccl_amd.synth_fill(send.data_ptr(), dt, n, op, SEED, 0) == 0
        assert dccl_amd.synth_fill(recv.data_ptr(), dt, n, op, SEED, 1) == 0
        assert dccl_amd.local_reduce(send.data_ptr(), recv.data_ptr(), dt, n, op) == 0
        got = recv.cpu().numpy().view(oracle.NP_DTYPES[dt])
        want = oracle.synth(n, dt, op, SEED, 1)
        assert oracle.expected_reduce(oracle.synth(n, dt, op, SEED, 0), want, dt, op) == 0
        assert got.tobytes() == want.tobytes(), (name, op)  # no NaN can arise from these operands
        del got, want
    assert dccl_amd.local_reduce(send.data_ptr(), recv.data_ptr(), dt, n, 4) == 5  # Avg: ncclInvalidUsage
