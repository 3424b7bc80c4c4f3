"""GPU parity tests: the HIP combine (through the C-ABI) against the oracle and the goldens.

Bar (DESIGN.md "Parity"): bit-exact for every integer dtype; for float dtypes bit-exact
too (0 ULP) except that a NaN output may carry any NaN payload.
Small sizes are checked element-by-element against the oracle restatement and the frozen
reference outputs; BASELINE sizes (1 GiB) against size-independent properties and torch's
own exact IEEE ops on the device.
"""
import json
import os

import numpy as np
import pytest

import oracle
from tests import ringsim
from tests.test_oracle import GOLDEN, fp_equal

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

ALL_DTYPES = list(range(10))
OPS = [0, 1, 2, 3]


@pytest.fixture(scope="module")
def dccl(gpu):
    import dccl_amd
    return dccl_amd


def dev_bytes(a: np.ndarray, offset: int = 0, device="cuda:0"):
    """Copy ``a`` to a fresh device allocation at ``offset`` bytes past a 256-B boundary.

    Returns (holder_tensor, device_address)."""
    raw = np.ascontiguousarray(a).view(np.uint8)
    t = torch.zeros(raw.size + offset + 256, dtype=torch.uint8, device=device)
    base = t.data_ptr()
    assert base % 256 == 0
    if raw.size:
        t[offset:offset + raw.size].copy_(torch.from_numpy(raw.copy()))
    return t, base + offset


def host_of(t, offset: int, like: np.ndarray) -> np.ndarray:
    nb = like.size * like.itemsize
    return t[offset:offset + nb].cpu().numpy().view(like.dtype)


def rand_inputs(rng, dt, n):
    npd = oracle.NP_DTYPES[dt]
    if dt in (6, 9):  # raw 16-bit patterns: every class (normals, denormals, inf, nan)
        s = rng.integers(0, 1 << 16, n, dtype=np.uint32).astype(np.uint16)
        r = rng.integers(0, 1 << 16, n, dtype=np.uint32).astype(np.uint16)
        return s, r
    if np.issubdtype(npd, np.integer):
        info = np.iinfo(npd)
        return (rng.integers(info.min, info.max, n, dtype=npd, endpoint=True),
                rng.integers(info.min, info.max, n, dtype=npd, endpoint=True))
    bits = np.uint32 if dt == 7 else np.uint64
    # random bit patterns hit denormals, infs and nans; mix with tame values
    s = rng.integers(0, np.iinfo(bits).max, n, dtype=bits, endpoint=True).view(npd)
    r = rng.integers(0, np.iinfo(bits).max, n, dtype=bits, endpoint=True).view(npd)
    tame = rng.random(n) < 0.5
    s[tame] = rng.standard_normal(int(tame.sum()))
    r[tame] = rng.standard_normal(int(tame.sum()))
    return s, r


def run_gpu(dccl, s: np.ndarray, r: np.ndarray, dt: int, op: int, soff=0, roff=0, stream=0):
    ts, ps = dev_bytes(s, soff)
    tr, pr = dev_bytes(r, roff)
    rc = dccl.local_reduce(ps, pr, dt, r.size, op, stream)
    torch.cuda.synchronize()
    return rc, host_of(tr, roff, r)


def expected(s, r, dt, op):
    return oracle.combine(s, r, dt, op)


# ----------------------------------------------------------------------------- goldens
@pytest.mark.parametrize("fixture", ["host_reduce_ref.npz", "host_reduce_half.npz"])
def test_golden_fixtures(dccl, fixture):
    z = np.load(os.path.join(GOLDEN, fixture))
    n_checked = 0
    for key in z.files:
        if not key.endswith("_out"):
            continue
        d, n, o, _ = key.split("_")
        dt, op = int(d[1:]), int(o[2:])
        rc, out = run_gpu(dccl, z[f"{d}_{n}_send"], z[f"{d}_{n}_recv"], dt, op)
        assert rc == 0
        assert fp_equal(out, z[key], dt), key
        n_checked += 1
    assert n_checked > 0


def test_return_codes(dccl):
    cases = json.load(open(os.path.join(GOLDEN, "rc_cases.json")))
    for c in cases:
        s = np.zeros(max(c["count"], 1), oracle.NP_DTYPES[c["dtype"]])
        rc, _ = run_gpu(dccl, s, s.copy(), c["dtype"], c["op"])
        # the reference fixture holds count=16; count=0 with a bad op is still rejected
        assert rc == c["rc"], c
    s = np.zeros(4, np.float32)
    assert run_gpu(dccl, s, s.copy(), 10, 0)[0] == 4   # unknown dtype: error, not silent (A.3 #4)
    assert run_gpu(dccl, s, s.copy(), -1, 0)[0] == 4
    assert dccl.local_reduce(0, 0, 7, 0, 0, 0) == 0    # empty
    assert dccl.local_reduce(0, 0, 7, 16, 0, 0) == 4   # null pointers with count > 0
    assert dccl.local_reduce(0, 0, 7, 0, 4, 0) == 5    # Avg rejected before the count shortcut


# ----------------------------------------------------------------------------- fuzz
@pytest.mark.parametrize("dt", ALL_DTYPES)
def test_fuzz_against_oracle(dccl, dt):
    rng = np.random.default_rng(100 + dt)
    for op in OPS:
        for n in [1, 2, 3, 15, 16, 17, 31, 255, 256, 257, 1023, 4096, 4099, 65537, 262147]:
            s, r = rand_inputs(rng, dt, n)
            rc, out = run_gpu(dccl, s, r, dt, op)
            assert rc == 0
            assert fp_equal(out, expected(s, r, dt, op), dt), (dt, op, n)


@pytest.mark.parametrize("dt", ALL_DTYPES)
def test_alignment_cases(dccl, dt):
    """Same 16-B phase (vector path with head/tail), different phases, non-element-aligned."""
    rng = np.random.default_rng(200 + dt)
    esz = np.dtype(oracle.NP_DTYPES[dt]).itemsize
    offsets = [(0, 0), (esz, esz), (3 * esz, 3 * esz), (0, esz), (esz, 0), (4 * esz, 0), (1, 1), (1, 3),
               (0, 1), (7, 5)]
    for soff, roff in offsets:
        for n in [1, 5, 33, 1000, 70001]:
            s, r = rand_inputs(rng, dt, n)
            op = int(rng.integers(0, 4))
            rc, out = run_gpu(dccl, s, r, dt, op, soff, roff)
            assert rc == 0
            assert fp_equal(out, expected(s, r, dt, op), dt), (dt, op, n, soff, roff)


@pytest.mark.parametrize("dt", ALL_DTYPES)
def test_shifted_kernel_every_phase(dccl, dt):
    """The shifted vector kernel (element-aligned operands, different 16-B phases): every phase
    difference the dtype allows, in both directions, sizes around the 64-vector tile (partial last
    tile, last lane's neighbour outside the tile), with head and tail scalars."""
    rng = np.random.default_rng(300 + dt)
    esz = np.dtype(oracle.NP_DTYPES[dt]).itemsize
    per_tile = 64 * (16 // esz)
    sizes = [1, 16 // esz + 1, per_tile - 1, per_tile + 16 // esz + 3, 3 * per_tile + 5, 40001]
    for p in range(esz, 16, esz):
        for soff, roff in ((p, 0), (0, p), (16 + p, 32 + esz if p + esz < 16 else 32)):
            if (soff - roff) % 16 == 0:
                continue
            for n in sizes:
                s, r = rand_inputs(rng, dt, n)
                op = int(rng.integers(0, 4))
                ts, ps = dev_bytes(s, soff)
                tr, pr = dev_bytes(r, roff)
                assert dccl.local_reduce(ps, pr, dt, n, op, 0) == 0
                torch.cuda.synchronize()
                assert fp_equal(host_of(tr, roff, r), expected(s, r, dt, op), dt), (dt, op, n, soff, roff)
                nb = n * esz  # nothing outside recv's bytes is written
                assert not tr[:roff].any() and not tr[roff + nb:].any(), (dt, n, soff, roff)


@pytest.mark.parametrize("dt", [2, 3, 4, 5, 6, 7, 8, 9])
def test_element_misaligned_every_offset(dccl, dt):
    """Element-misaligned operands (recv not a multiple of sizeof(T); reduce_unaligned_kernel, 16-B accesses
    at any byte address, and its element-wise tail): every recv byte offset in a 16-B vector, send at several byte phases, sizes around a 64-vector tile,
    partial tiles; nothing outside recv's bytes is written."""
    rng = np.random.default_rng(700 + dt)
    esz = np.dtype(oracle.NP_DTYPES[dt]).itemsize
    per_tile = 64 * (16 // esz)
    sizes = [1, 2, 16 // esz + 1, per_tile - 1, per_tile, per_tile + 1, 2 * per_tile + 16 // esz + 3, 40001]
    for roff in range(1, 16):
        if roff % esz == 0:
            continue
        for soff in sorted({0, roff, (roff + 3) % 16, 16 - roff, 1 + 16 * (roff % 3)}):
            for n in sizes:
                s, r = rand_inputs(rng, dt, n)
                op = int(rng.integers(0, 4))
                ts, ps = dev_bytes(s, soff)
                tr, pr = dev_bytes(r, roff)
                assert dccl.local_reduce(ps, pr, dt, n, op, 0) == 0
                torch.cuda.synchronize()
                assert fp_equal(host_of(tr, roff, r), expected(s, r, dt, op), dt), (dt, op, n, soff, roff)
                nb = n * esz
                assert not tr[:roff].any() and not tr[roff + nb:].any(), (dt, n, soff, roff)


@pytest.mark.parametrize("dt", [2, 3, 4, 5, 6, 7, 8, 9])
def test_send_byte_misaligned_every_offset(dccl, dt):
    """A send at any byte address against an element-aligned recv (the shifted kernel with a byte phase, send's
    head / tail elements read bytewise): every send byte offset that is not a multiple of sizeof(T), recv in
    and off its 16-B and 128-B grids, sizes around a 64-vector tile; nothing outside recv's bytes is written."""
    rng = np.random.default_rng(900 + dt)
    esz = np.dtype(oracle.NP_DTYPES[dt]).itemsize
    per_tile = 64 * (16 // esz)
    sizes = [1, 2, 16 // esz + 1, per_tile - 1, per_tile + 1, 2 * per_tile + 16 // esz + 3, 40001]
    for soff in range(1, 32):
        if soff % esz == 0:
            continue
        for roff in (0, esz, 48, 128 - esz):
            for n in sizes:
                s, r = rand_inputs(rng, dt, n)
                op = int(rng.integers(0, 4))
                ts, ps = dev_bytes(s, soff)
                tr, pr = dev_bytes(r, roff)
                assert dccl.local_reduce(ps, pr, dt, n, op, 0) == 0
                torch.cuda.synchronize()
                assert fp_equal(host_of(tr, roff, r), expected(s, r, dt, op), dt), (dt, op, n, soff, roff)
                nb = n * esz
                assert not tr[:roff].any() and not tr[roff + nb:].any(), (dt, n, soff, roff)


@pytest.mark.parametrize("dt", [6, 9])
def test_all_16bit_patterns(dccl, dt):
    """Every fp16 / bf16 bit pattern as recv against a fixed set of partners."""
    r_all = np.arange(1 << 16, dtype=np.uint32).astype(np.uint16)
    partners = np.array([0x0000, 0x8000, 0x0001, 0x3C00 if dt == 6 else 0x3F80, 0x7BFF if dt == 6 else 0x7F7F,
                         0x7C00 if dt == 6 else 0x7F80, 0x7E00 if dt == 6 else 0x7FC0, 0xC000, 0x03FF], np.uint16)
    for p in partners:
        s = np.full_like(r_all, p)
        for op in OPS:
            rc, out = run_gpu(dccl, s, r_all, dt, op)
            assert rc == 0
            assert fp_equal(out, expected(s, r_all, dt, op), dt), (dt, op, hex(int(p)))


@pytest.mark.parametrize("off", [0, 1, 3, 6, 16])
def test_aliasing_send_is_recv(dccl, off):
    """send == recv (allowed by the boundary), element-aligned or not: every kernel's lane only uses the
    bytes of its own elements, so in-place doubling / squaring is exact across tiles and waves."""
    rng = np.random.default_rng(5 + off)
    for dt in ALL_DTYPES:
        for n in (10007, 200003):
            s, _ = rand_inputs(rng, dt, n)
            t, p = dev_bytes(s, off)
            for op in OPS:
                assert dccl.local_reduce(p, p, dt, s.size, op, 0) == 0
                torch.cuda.synchronize()
                got = host_of(t, off, s)
                assert fp_equal(got, expected(s, s, dt, op), dt), (dt, n, op, off)
                s = got.copy()
            assert not t[:off].any() and not t[off + s.nbytes:].any()


@pytest.mark.parametrize("entry", ["pair", "multi", "chain_src", "chain_own", "host", "chain_host", "copy"])
def test_partial_overlap_contract(dccl, entry):
    """VERDICT r5 item 2, on the GPU: every combine entry point returns ncclInvalidArgument for an operand
    overlapping the destination by one element (either direction) and leaves the destination untouched; the
    same operands one element further apart (adjacent, no shared byte) combine bit-exactly against the
    oracle."""
    dt, n, op = 7, 4099, 0
    esz = 4
    rng = np.random.default_rng(77)
    host = entry in ("host", "chain_host")
    dev = "cpu" if host else "cuda"
    for sh in (-(n - 1), n - 1, -n, n):  # elements between the destination's start and the operand's
        buf = torch.zeros(3 * n, dtype=torch.float32, device=dev)
        if host:
            buf = buf.pin_memory()
        vals = rng.standard_normal(3 * n).astype(np.float32)
        buf.copy_(torch.from_numpy(vals))
        other = torch.from_numpy(rng.standard_normal(n).astype(np.float32)).to(dev)
        if host:
            other = other.pin_memory()
        d0 = n  # destination: elements [n, 2n)
        dptr, optr = buf.data_ptr() + d0 * esz, buf.data_ptr() + (d0 + sh) * esz
        before = buf.cpu().numpy().copy()
        if entry == "pair":
            rc = dccl.local_reduce(optr, dptr, dt, n, op, 0)
        elif entry == "multi":
            rc = dccl.local_reduce_multi([other.data_ptr(), optr], dptr, dt, n, op, 0)
        elif entry == "chain_src":
            rc = dccl.local_reduce_chain([other.data_ptr(), optr], other.data_ptr(), dptr, dt, n, op, 0)
        elif entry == "chain_own":
            rc = dccl.local_reduce_chain([other.data_ptr()], optr, dptr, dt, n, op, 0)
        elif entry == "host":
            rc = dccl.local_reduce_host(optr, dptr, dt, n, op)
        elif entry == "chain_host":
            rc = dccl.local_reduce_chain_host([other.data_ptr()], optr, dptr, dt, n, op)
        else:
            rc = dccl.copy_multi([optr], [dptr], n * esz, 0)
        torch.cuda.synchronize()
        after = buf.cpu().numpy()
        if abs(sh) < n:
            assert rc == 4, (entry, sh, rc)
            assert after.tobytes() == before.tobytes(), (entry, sh)
            continue
        assert rc == 0, (entry, sh, rc)
        src = before[d0 + sh:d0 + sh + n]
        o = other.cpu().numpy()
        if entry in ("pair", "host"):
            want = oracle.combine(src, before[d0:d0 + n], dt, op)
        elif entry == "multi":
            want = oracle.combine(src, oracle.combine(o, before[d0:d0 + n], dt, op), dt, op)
        elif entry == "chain_src":  # dst = op(own, op(s1, s0)), own = s0 = other
            want = oracle.combine(oracle.combine(o, src, dt, op), o, dt, op)
        elif entry in ("chain_own", "chain_host"):  # dst = op(own, s0)
            want = oracle.combine(o, src, dt, op)
        else:
            want = src
        assert fp_equal(after[d0:d0 + n], want, dt), (entry, sh)
        rest = np.concatenate([after[:d0], after[d0 + n:]]), np.concatenate([before[:d0], before[d0 + n:]])
        assert rest[0].tobytes() == rest[1].tobytes(), (entry, sh)


def test_stream_ordering(dccl):
    """Launches on a user stream are ordered behind prior work on that stream."""
    st = torch.cuda.Stream()
    n = 1 << 22
    with torch.cuda.stream(st):
        a = torch.ones(n, device="cuda", dtype=torch.float32)
        b = torch.full((n,), 2.0, device="cuda", dtype=torch.float32)
        for _ in range(10):
            assert dccl.local_reduce(b.data_ptr(), a.data_ptr(), 7, n, 0, st.cuda_stream) == 0
    st.synchronize()
    assert torch.all(a == 21.0)


# ----------------------------------------------------------------------------- k-way
@pytest.mark.parametrize("k", [1, 2, 3, 5, 8])
def test_multi_matches_sequential(dccl, k):
    rng = np.random.default_rng(300 + k)
    for dt in ALL_DTYPES:
        for n, off in [(1, 0), (17, 0), (4099, 0), (100003, 0), (1000, 1)]:
            op = int(rng.integers(0, 4))
            sends = [rand_inputs(rng, dt, n)[0] for _ in range(k)]
            _, r = rand_inputs(rng, dt, n)
            holders = [dev_bytes(x, off) for x in sends]
            tr, pr = dev_bytes(r, off)
            assert dccl.local_reduce_multi([h[1] for h in holders], pr, dt, n, op, 0) == 0
            torch.cuda.synchronize()
            want = r
            for x in sends:
                want = expected(x, want, dt, op)
            assert fp_equal(host_of(tr, off, r), want, dt), (k, dt, n, op)
    assert dccl.local_reduce_multi([], 0, 7, 4, 0, 0) == 4


@pytest.mark.parametrize("k", [1, 2, 3, 4, 7, 8])
def test_multi_mixed_phases(dccl, k):
    """Element-aligned sources at their own 16-B and 128-B phases (the phased k-way kernel)."""
    rng = np.random.default_rng(400 + k)
    for dt in ALL_DTYPES:
        esz = int(oracle.NP_DTYPES[dt]().itemsize)
        for n in (1, 5, 63, 4099, 65539):
            op = int(rng.integers(0, 4))
            sends = [rand_inputs(rng, dt, n)[0] for _ in range(k)]
            _, r = rand_inputs(rng, dt, n)
            offs = [int(rng.integers(0, 256 // esz)) * esz for _ in range(k)]
            offs[0] = (offs[0] // 16) * 16 + (esz if esz < 16 else 0)  # at least one source off 16-B phase
            roff = int(rng.integers(0, 256 // esz)) * esz
            holders = [dev_bytes(x, o) for x, o in zip(sends, offs)]
            tr, pr = dev_bytes(r, roff)
            assert dccl.local_reduce_multi([h[1] for h in holders], pr, dt, n, op, 0) == 0
            torch.cuda.synchronize()
            want = r
            for x in sends:
                want = expected(x, want, dt, op)
            assert fp_equal(host_of(tr, roff, r), want, dt), (k, dt, n, op, offs, roff)


@pytest.mark.parametrize("k", [2, 3, 5, 8])
def test_multi_byte_offsets(dccl, k):
    """Sources at any byte address (phased kernel with byte phases, sources' head / tail read bytewise) and
    recv at any byte address (reduce_windows_kernel when recv is not element-aligned): every dtype
    wider than a byte, sizes around a tile, against the sequential oracle; nothing outside recv written."""
    rng = np.random.default_rng(1300 + k)
    for dt in [2, 3, 4, 5, 6, 7, 8, 9]:
        esz = int(oracle.NP_DTYPES[dt]().itemsize)
        per_tile = 64 * (16 // esz)
        for n in (1, 16 // esz + 1, per_tile - 1, per_tile + 3, 2 * per_tile + 5, 40001):
            for recv_mis in (False, True):
                op = int(rng.integers(0, 4))
                sends = [rand_inputs(rng, dt, n)[0] for _ in range(k)]
                _, r = rand_inputs(rng, dt, n)
                offs = [int(rng.integers(0, 64)) for _ in range(k)]
                offs[0] = offs[0] // esz * esz + 1  # at least one source not element-aligned
                roff = int(rng.integers(0, 64 // esz)) * esz
                if recv_mis:
                    roff += int(rng.integers(1, esz))
                holders = [dev_bytes(x, o) for x, o in zip(sends, offs)]
                tr, pr = dev_bytes(r, roff)
                assert dccl.local_reduce_multi([h[1] for h in holders], pr, dt, n, op, 0) == 0
                torch.cuda.synchronize()
                want = r
                for x in sends:
                    want = expected(x, want, dt, op)
                assert fp_equal(host_of(tr, roff, r), want, dt), (k, dt, n, op, offs, roff)
                nb = n * esz
                assert not tr[:roff].any() and not tr[roff + nb:].any(), (k, dt, n, offs, roff)


@pytest.mark.parametrize("k", [1, 2, 3, 5, 8])
def test_misaligned_destination_tile_orders(dccl, k):
    """A destination that is not element-aligned, with sources at 16-B phase 0 (the kernels take the group-
    interleaved order for k <= 2 and block order above, reduce_kernels.hpp tile_order) and at phase 4 (XCD
    ranges), k-way and chain (own = dst, in place), at tile counts below one group of 64, exactly two groups,
    and several groups plus a partial one: every element against the oracle applied in order (k-way) and in
    the ring's chain order, nothing outside the destination written."""
    rng = np.random.default_rng(1700 + k)
    for dt in (7, 9, 4):
        esz = int(oracle.NP_DTYPES[dt]().itemsize)
        per_tile = 64 * (16 // esz)
        for n in (per_tile * 5 + 3, per_tile * 128, per_tile * 200 + 7):
            for src_phase in (0, 4):
                op = int(rng.integers(0, 4))
                sends = [rand_inputs(rng, dt, n)[0] for _ in range(k)]
                _, r = rand_inputs(rng, dt, n)
                holders = [dev_bytes(x, 16 * j + src_phase) for j, x in enumerate(sends)]
                roff = 32 + 1 + int(rng.integers(0, esz - 1))
                # k-way (k = 1 is the pairwise kernel)
                tr, pr = dev_bytes(r, roff)
                rc = dccl.local_reduce(holders[0][1], pr, dt, n, op, 0) if k == 1 else \
                    dccl.local_reduce_multi([h[1] for h in holders], pr, dt, n, op, 0)
                assert rc == 0
                torch.cuda.synchronize()
                want = r
                for x in sends:
                    want = expected(x, want, dt, op)
                assert fp_equal(host_of(tr, roff, r), want, dt), ("multi", k, dt, n, op, src_phase, roff)
                assert not tr[:roff].any() and not tr[roff + n * esz:].any()
                # chain, in place: dst = op(own, op(s[k-1], ... op(s[1], s[0])))
                to, po = dev_bytes(r, roff)
                assert dccl.local_reduce_chain([h[1] for h in holders], po, po, dt, n, op, 0) == 0
                torch.cuda.synchronize()
                acc = sends[0]
                for x in sends[1:]:
                    acc = expected(acc, x, dt, op)
                want_c = expected(acc, r, dt, op)
                assert fp_equal(host_of(to, roff, r), want_c, dt), ("chain", k, dt, n, op, src_phase, roff)
                assert not to[:roff].any() and not to[roff + n * esz:].any()


def _torch_op(op):
    return {0: torch.add, 1: torch.mul, 2: torch.maximum, 3: torch.minimum}[op]


@pytest.mark.parametrize("mib", [64, 72, 96])
@pytest.mark.parametrize("k", [3, 4, 5, 6, 7, 8])
def test_windows_tuned_forms_full_size(dccl, k, mib):
    """From caps::kWindowTunedBytes (96 MiB per operand) reduce_windows_kernel takes its tuned forms (caps.hpp
    kWindow: block order under a 26-wave cap with sources in phase; with sources off phase group order, loads-
    first at k = 4, 5 under 14 / 12 waves, loads-first in runs of 4 tiles at k = 6..8) and takes over the phased
    launches at k-way k = 3..5 and chain k = 4..7; at 64 and 72 MiB (caps.hpp window_mid) sources off phase take
    the mid-size form, phased launches into a 16-B aligned destination too, in-phase sources the per-operand
    form uncapped.  Destination not
    element-aligned, and element-aligned at 16-B phases 0 and 4; sources at phase 0, 4 and 16; k-way and chain in
    place; fp32 Sum, int32 Max, bf16 Sum, int64 Min, against torch applied on the device in the kernels' order, bit for
    bit; nothing outside the destination written."""
    nb = (mib << 20) + 4096
    for dt, tdt, ibits, op in [(7, torch.float32, torch.int32, 0), (2, torch.int32, torch.int32, 2),
                               (9, torch.bfloat16, torch.int16, 0), (4, torch.int64, torch.int64, 3)]:
        esz = torch.empty(0, dtype=tdt).element_size()
        n = nb // esz
        mis = 1 if esz == 2 else 2
        g = torch.Generator(device="cuda").manual_seed(2400 + k + dt)

        def operand():
            if tdt in (torch.int32, torch.int64):
                return torch.randint(-(1 << 30), 1 << 30, (n,), device="cuda", dtype=tdt, generator=g)
            return (torch.rand(n, device="cuda", generator=g) * 2 - 1).to(tdt)

        def placed(x, off):
            buf = torch.zeros(nb + 1024, dtype=torch.uint8, device="cuda")
            buf[off:off + nb].copy_(x.view(torch.uint8))
            return buf

        f = _torch_op(op)
        for roff, soff in [(mis, 0), (mis, 4), (0, 4), (4, 0), (0, 16)]:
            sends = [operand() for _ in range(k)]
            r = operand()
            sbufs = [placed(x, 64 * (j + 1) + soff) for j, x in enumerate(sends)]
            sptrs = [b.data_ptr() + 64 * (j + 1) + soff for j, b in enumerate(sbufs)]
            want_m = r
            for x in sends:
                want_m = f(want_m, x)
            acc = sends[0]
            for x in sends[1:]:
                acc = f(x, acc)
            want_c = f(r, acc)
            for form, want in (("multi", want_m), ("chain", want_c)):
                d = placed(r, roff)
                p = d.data_ptr() + roff
                rc = dccl.local_reduce_multi(sptrs, p, dt, n, op, 0) if form == "multi" else \
                    dccl.local_reduce_chain(sptrs, p, p, dt, n, op, 0)
                assert rc == 0
                torch.cuda.synchronize()
                got = d[roff:roff + nb].clone().view(tdt)
                assert torch.equal(got.view(ibits), want.view(ibits)), (form, k, dt, roff, soff)
                assert not d[:roff].any() and not d[roff + nb:].any(), (form, k, dt, roff, soff)
                del d
            del sbufs, sends
        torch.cuda.empty_cache()


@pytest.mark.parametrize("k", [4, 7])
def test_chain_own_only_off_phase_full_size(dccl, k):
    """A chain whose sources share the destination's 16-B phase while `own` sits at another phase (own != dst),
    at 96 MiB per operand, where the phased chain launches with sources off phase take reduce_windows_kernel:
    this one keeps the phased kernels (the windows forms were measured with sources off phase).
    fp32 Sum and int32 Max against torch in the ring's order, bit for bit; nothing outside dst written."""
    nb = (96 << 20) + 4096
    for dt, tdt, op in [(7, torch.float32, 0), (2, torch.int32, 2)]:
        n = nb // 4
        g = torch.Generator(device="cuda").manual_seed(3100 + k + dt)

        def operand():
            if tdt == torch.int32:
                return torch.randint(-(1 << 30), 1 << 30, (n,), device="cuda", dtype=tdt, generator=g)
            return torch.rand(n, device="cuda", generator=g) * 2 - 1

        sends = [operand() for _ in range(k)]
        own = operand()
        obuf = torch.zeros(nb + 1024, dtype=torch.uint8, device="cuda")
        obuf[4:4 + nb].copy_(own.view(torch.uint8))
        d = torch.zeros(nb + 1024, dtype=torch.uint8, device="cuda")
        f = _torch_op(op)
        acc = sends[0]
        for x in sends[1:]:
            acc = f(x, acc)
        want = f(own, acc)
        rc = dccl.local_reduce_chain([x.data_ptr() for x in sends], obuf.data_ptr() + 4, d.data_ptr(), dt, n, op, 0)
        assert rc == 0
        torch.cuda.synchronize()
        assert torch.equal(d[:nb].view(torch.int32), want.view(torch.int32)), (k, dt)
        assert not d[nb:].any()
        del sends, own, obuf, d
        torch.cuda.empty_cache()


# ----------------------------------------------------------------------------- host path
@pytest.mark.parametrize("zero_copy", ["default", "0"])
@pytest.mark.parametrize("pinned", ["none", "both", "send"])
def test_host_staged(dccl, pinned, zero_copy, monkeypatch):
    """Host operands: zero-copy kernel (page-locked, or pageable <= 16 MiB bounced) and the
    3-stream DMA pipeline (large pageable, or DCCL_HOST_ZEROCOPY_MAX=0).  "send" is Derecho's
    shape: a registered RDMA scratchpad combined into a pageable user chunk."""
    if zero_copy == "0":
        monkeypatch.setenv("DCCL_HOST_ZEROCOPY_MAX", "0")
    rng = np.random.default_rng(400)
    for dt in [0, 6, 7, 8, 9, 4]:
        # the last size spans > 3 DMA staging slots of 16 MiB for 4-B types
        for n in [1, 1000, 65537, (16 << 20) // 4 + 1, 3 * (16 << 20) // 4 + 12345]:
            s, r = rand_inputs(rng, dt, n)
            op = int(rng.integers(0, 4))
            want = expected(s, r, dt, op)
            s2, r2 = s.copy(), r.copy()
            regs = {"none": [], "both": [s2, r2], "send": [s2]}[pinned]
            for x in regs:
                assert dccl.register_host_memory(x.ctypes.data, x.nbytes) == 0
            try:
                assert dccl.local_reduce_host(s2.ctypes.data, r2.ctypes.data, dt, n, op) == 0
            finally:
                for x in regs:
                    dccl.deregister_host_memory(x.ctypes.data)
            assert fp_equal(r2, want, dt), (dt, n, op)
            assert s2.tobytes() == s.tobytes()


@pytest.mark.parametrize("pinned", [False, True])
def test_host_staged_byte_offsets(dccl, pinned):
    """Host operands that are not element-aligned: registered (the zero-copy kernel reads them through their
    device alias at the same byte offsets, so the shifted / misaligned-recv kernels run over PCIe) and
    pageable (bounced into aligned staging slots); sizes on both sides of the zero-copy limit."""
    rng = np.random.default_rng(402)
    for dt, n in [(7, 1000), (7, (16 << 20) // 4 + 3), (8, 4099), (6, (1 << 20) + 1), (4, 3 * (16 << 20) // 8 + 7)]:
        esz = np.dtype(oracle.NP_DTYPES[dt]).itemsize
        for soff, roff in ((1, 0), (0, 1), (3, esz // 2 + 1)):
            s, r = rand_inputs(rng, dt, n)
            op = int(rng.integers(0, 4))
            want = expected(s, r, dt, op)
            sb = np.zeros(s.nbytes + 64, dtype=np.uint8)
            rb = np.zeros(r.nbytes + 64, dtype=np.uint8)
            sb[soff:soff + s.nbytes] = s.view(np.uint8)
            rb[roff:roff + r.nbytes] = r.view(np.uint8)
            regs = [sb, rb] if pinned else []
            for x in regs:
                assert dccl.register_host_memory(x.ctypes.data, x.nbytes) == 0
            try:
                assert dccl.local_reduce_host(sb.ctypes.data + soff, rb.ctypes.data + roff, dt, n, op) == 0
            finally:
                for x in regs:
                    dccl.deregister_host_memory(x.ctypes.data)
            got = rb[roff:roff + r.nbytes].view(r.dtype)
            assert fp_equal(got, want, dt), (pinned, dt, n, op, soff, roff)
            assert not rb[:roff].any() and not rb[roff + r.nbytes:].any()
            assert sb[soff:soff + s.nbytes].tobytes() == s.tobytes()


ZERO_COPY_CAP_CHILD = r"""
import sys
import numpy as np
import torch
sys.path.insert(0, sys.argv[1])
import dccl_amd, oracle
from tests.test_gpu_parity import rand_inputs, expected
from tests.test_oracle import fp_equal
torch.cuda.set_device(0)
rng = np.random.default_rng(404)
bad = []
# every pairwise kernel class over PCIe (aligned, line-straddling, shifted, byte-shifted send, misaligned recv),
# sizes with a partial last tile, head and tail scalars, and many tiles per striding wave
for dt, n, soff, roff in [(7, 3 * 65536 + 5, 0, 0), (7, 70001, 64, 0), (7, 70001, 4, 0), (2, 50003, 1, 0),
                          (8, 40001, 0, 3), (6, 90001, 2, 6), (0, 300007, 5, 0)]:
    s, r = rand_inputs(rng, dt, n)
    op = int(rng.integers(0, 4))
    want = expected(s, r, dt, op)
    sb = np.zeros(s.nbytes + 256, np.uint8); rb = np.zeros(r.nbytes + 256, np.uint8)
    sb[soff:soff + s.nbytes] = s.view(np.uint8); rb[roff:roff + r.nbytes] = r.view(np.uint8)
    for x in (sb, rb):
        assert dccl_amd.register_host_memory(x.ctypes.data, x.nbytes) == 0
    rc = dccl_amd.local_reduce_host(sb.ctypes.data + soff, rb.ctypes.data + roff, dt, n, op)
    for x in (sb, rb):
        dccl_amd.deregister_host_memory(x.ctypes.data)
    got = rb[roff:roff + r.nbytes].view(r.dtype)
    if rc != 0 or not fp_equal(got, want, dt) or rb[:roff].any() or rb[roff + r.nbytes:].any():
        bad.append(("pair", dt, n, soff, roff, rc))
# the host chain combine, staged (pageable) and in place on registered operands
for dt, n, k in [(7, 200003, 3), (4, 100001, 7), (9, 150001, 1)]:
    srcs = [rand_inputs(rng, dt, n)[0] for _ in range(k)]
    own = rand_inputs(rng, dt, n)[0]
    op = int(rng.integers(0, 4))
    want = srcs[0].copy()
    for j in range(1, k):
        want = expected(want, srcs[j], dt, op)
    want = expected(want, own, dt, op)
    for registered in (False, True):
        o = own.copy()
        regs = srcs + [o] if registered else []
        for x in regs:
            assert dccl_amd.register_host_memory(x.ctypes.data, x.nbytes) == 0
        rc = dccl_amd.local_reduce_chain_host([x.ctypes.data for x in srcs], o.ctypes.data, o.ctypes.data, dt, n, op)
        for x in regs:
            dccl_amd.deregister_host_memory(x.ctypes.data)
        if rc != 0 or not fp_equal(o, want, dt):
            bad.append(("chain", dt, n, k, registered, rc))
print("BAD", bad)
sys.exit(1 if bad else 0)
"""


@pytest.mark.parametrize("waves", ["8", "512", "0"])
def test_host_zero_copy_wave_caps(waves):
    """The zero-copy host combines under their wave caps (DCCL_HOST_ZEROCOPY_WAVES / DCCL_HOST_CHAIN_WAVES, read
    once per process, so each cap runs in a child): 8 waves (hundreds of tiles per striding wave), the default
    512 and none; every pairwise kernel class and the chain, bit-exact against the oracle, nothing written
    outside the destination."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {**os.environ, "DCCL_HOST_ZEROCOPY_WAVES": waves, "DCCL_HOST_CHAIN_WAVES": waves, "PYTHONPATH": root}
    p = subprocess.run([sys.executable, "-c", ZERO_COPY_CAP_CHILD, root], env=env, capture_output=True, text=True,
                       timeout=240)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-3000:])


@pytest.mark.parametrize("threads", ["1", "3", "8"])
def test_host_staged_copy_threads(dccl, threads, monkeypatch):
    """Pageable bounce copies split over DCCL_HOST_COPY_THREADS threads: odd byte counts, every slice
    boundary, pipeline and zero-copy sizes (the pool is created per thread, so run in a fresh thread)."""
    import threading
    monkeypatch.setenv("DCCL_HOST_COPY_THREADS", threads)
    rng = np.random.default_rng(401)
    errors = []

    def body():
        try:
            torch.cuda.set_device(0)
            for dt, n in [(0, (1 << 20) + 7), (7, (3 << 20) + 5), (8, 5 * (1 << 20) + 3), (6, 9 * (1 << 20) + 1)]:
                s, r = rand_inputs(rng, dt, n)
                op = int(rng.integers(0, 4))
                want = expected(s, r, dt, op)
                r2 = r.copy()
                assert dccl.local_reduce_host(s.ctypes.data, r2.ctypes.data, dt, n, op) == 0
                assert fp_equal(r2, want, dt), (threads, dt, n, op)
        except Exception as e:  # surfaced in the test thread
            errors.append(e)

    t = threading.Thread(target=body)
    t.start()
    t.join()
    assert not errors, errors


# ----------------------------------------------------------------------------- ring (C1)
@pytest.mark.parametrize("kind", ["float32", "uint32"])
def test_c1_ring_goldens_on_gpu(dccl, kind):
    g = json.load(open(os.path.join(GOLDEN, "c1_ring.json")))
    W, n = g["world_size"], g["count"]
    dt = 7 if kind == "float32" else 3
    bufs = [torch.full((n * 4,), r, dtype=torch.uint8, device="cuda").view(torch.int32) for r in range(W)]

    def combine(send, recv):
        assert dccl.local_reduce(send.data_ptr(), recv.data_ptr(), dt, recv.numel(), 0, 0) == 0

    def copy(dst, src):
        dst.copy_(src)

    done = 0
    for target in sorted(int(k) for k in g[kind]):
        while done < target:
            ringsim.ring_allreduce(bufs, combine, copy)
            done += 1
        torch.cuda.synchronize()
        want = int(g[kind][str(target)], 16)
        for b in bufs:
            got = b.cpu().numpy().view(np.uint32)
            assert np.all(got == want), (kind, target, hex(int(got[0])))


# ----------------------------------------------------------------------------- full size
def _torch_expected(r, s, op):
    if op == 0:
        return r + s
    if op == 1:
        return r * s
    if op == 2:
        return torch.where(r < s, s, r)
    return torch.where(r > s, s, r)


@pytest.mark.slow
@pytest.mark.parametrize("dt,tdt", [(7, "float32"), (6, "float16"), (9, "bfloat16"), (2, "int32"),
                                    (4, "int64"), (0, "int8"), (1, "uint8"), (8, "float64")])
def test_one_gib_against_torch(dccl, dt, tdt):
    """BASELINE config C3 sizes (1 GiB per operand): every op, bit-exact vs torch's device ops."""
    tdtype = getattr(torch, tdt)
    esz = torch.empty(0, dtype=tdtype).element_size()
    n = (1 << 30) // esz
    g = torch.Generator(device="cuda").manual_seed(dt)
    if tdtype.is_floating_point:
        s = torch.rand(n, device="cuda", generator=g, dtype=torch.float32).mul_(2).sub_(1).to(tdtype)
        r0 = torch.rand(n, device="cuda", generator=g, dtype=torch.float32).mul_(2).sub_(1).to(tdtype)
    else:
        info = torch.iinfo(tdtype)
        s = torch.randint(info.min, info.max, (n,), device="cuda", generator=g, dtype=tdtype)
        r0 = torch.randint(info.min, info.max, (n,), device="cuda", generator=g, dtype=tdtype)
    for op in OPS:
        r = r0.clone()
        assert dccl.local_reduce(s.data_ptr(), r.data_ptr(), dt, n, op, 0) == 0
        want = _torch_expected(r0, s, op)
        if tdtype.is_floating_point:
            nan_r, nan_w = torch.isnan(r), torch.isnan(want)
            assert torch.equal(nan_r, nan_w)
            bits = {2: torch.int16, 4: torch.int32, 8: torch.int64}[esz]
            assert torch.equal(r.view(bits)[~nan_r], want.view(bits)[~nan_w]), op
        else:
            assert torch.equal(r, want), op
        del r, want
    torch.cuda.empty_cache()


@pytest.mark.slow
def test_one_gib_inverse_roundtrip(dccl):
    """Size-independent property at 1 GiB: int32 Sum with s then with -s restores recv exactly."""
    n = (1 << 30) // 4
    g = torch.Generator(device="cuda").manual_seed(9)
    r0 = torch.randint(-2**31, 2**31 - 1, (n,), device="cuda", generator=g, dtype=torch.int32)
    s = torch.randint(-2**31, 2**31 - 1, (n,), device="cuda", generator=g, dtype=torch.int32)
    r = r0.clone()
    assert dccl.local_reduce(s.data_ptr(), r.data_ptr(), 2, n, 0, 0) == 0
    s.neg_()
    assert dccl.local_reduce(s.data_ptr(), r.data_ptr(), 2, n, 0, 0) == 0
    assert torch.equal(r, r0)


@pytest.mark.slow
def test_grid_stride_past_launch_cap(dccl):
    """Maximum-size edge of the launch arithmetic: the vector kernel's grid is capped at 2^24 one-wave
    blocks (16 GiB of 16-B vectors per operand), beyond which blocks stride.  17 GiB + 37 B uint8
    operands at a 5-B offset (scalar head and tail, a partial last tile, > 1 tile per block), Sum,
    checked 1 GiB at a time against torch's wrapping uint8 add; bytes before the operands untouched."""
    off, n = 5, (17 << 30) + 37
    free, _ = torch.cuda.mem_get_info()
    if free < 3 * (n + off) + (4 << 30):
        pytest.skip("needs ~56 GiB of free HBM")
    g = torch.Generator(device="cuda").manual_seed(17)
    sb = torch.empty(n + off, dtype=torch.uint8, device="cuda").random_(0, 256, generator=g)
    rb = torch.empty(n + off, dtype=torch.uint8, device="cuda").random_(0, 256, generator=g)
    r0 = rb.clone()
    try:
        assert dccl.local_reduce(sb.data_ptr() + off, rb.data_ptr() + off, 1, n, 0, 0) == 0
        torch.cuda.synchronize()
        assert torch.equal(rb[:off], r0[:off])
        step = 1 << 30
        for a in range(off, n + off, step):
            b = min(a + step, n + off)
            assert torch.equal(rb[a:b], r0[a:b] + sb[a:b]), a
    finally:
        del sb, rb, r0
        torch.cuda.empty_cache()


def test_misaligned_reference_wrong_build_correct(dccl):
    """SURVEY.md A.4 fixtures: at the reference's own misaligned recv offsets the HIP combine gives the
    element-wise result and touches nothing past `count`; the reference's output differs."""
    from tests.test_oracle import _misaligned_cases
    for i, dt, off, n, s, r, ref, correct in _misaligned_cases():
        ts, ps = dev_bytes(s, off)
        tr, pr = dev_bytes(r, off)
        assert dccl.local_reduce(ps, pr, dt, n, 0, 0) == 0
        torch.cuda.synchronize()
        got = host_of(tr, off, r)
        assert got.tobytes() == correct.tobytes(), i


def test_concurrent_threads_and_streams(dccl):
    """Reentrancy (SURVEY §8(b) threading): 6 host threads, each with its own stream, run the device combine
    (pairwise at several alignments, k-way, chain) and the host-staged combine concurrently on their own
    buffers, 20 times each; every result matches the sequential expectation."""
    import threading
    errors = []

    def worker(seed):
        try:
            torch.cuda.set_device(0)
            rng = np.random.default_rng(900 + seed)
            st = torch.cuda.Stream()
            n = 100_003 + seed
            for it in range(20):
                dt = [2, 7, 9, 4][(seed + it) % 4]
                op = int(rng.integers(0, 4))
                s, r = rand_inputs(rng, dt, n)
                soff, roff = [(0, 0), (4, 0), (1, 0), (0, 2)][it % 4]
                if dt == 4:
                    soff, roff = soff * 2, 0
                if dt == 9 and roff:
                    roff = 1
                ts, ps = dev_bytes(s, soff)
                tr, pr = dev_bytes(r, roff)
                torch.cuda.current_stream().synchronize()  # the operand copies ran on this thread's default stream
                with torch.cuda.stream(st):
                    if it % 5 == 4:  # the host-staged path on this thread's own staging resources
                        s2, r2 = s.copy(), r.copy()
                        assert dccl.local_reduce_host(s2.ctypes.data, r2.ctypes.data, dt, n, op) == 0
                        assert fp_equal(r2, expected(s, r, dt, op), dt), ("host", seed, it)
                        continue
                    if it % 3 == 2:
                        assert dccl.local_reduce_multi([ps, ps], pr, dt, n, op, st.cuda_stream) == 0
                        want = expected(s, expected(s, r, dt, op), dt, op)
                    else:
                        assert dccl.local_reduce(ps, pr, dt, n, op, st.cuda_stream) == 0
                        want = expected(s, r, dt, op)
                    st.synchronize()
                assert fp_equal(host_of(tr, roff, r), want, dt), (seed, it, dt, op, soff, roff)
        except Exception as e:  # surfaced in the test thread
            errors.append(e)

    threads = [threading.Thread(target=worker, args=(i,)) for i in range(6)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(120)
    assert not any(t.is_alive() for t in threads), "a worker hung"
    assert not errors, errors[:2]


def test_graph_capture_replay(dccl):
    """dccl_local_reduce only enqueues a kernel on the given stream, so it can be captured in a HIP
    graph (torch.cuda.graph) and replayed; each replay applies the combine once more."""
    n = (1 << 20) + 3
    s = torch.full((n,), 1.0, device="cuda")
    r = torch.zeros(n, device="cuda")
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=st):
            for _ in range(4):
                assert dccl.local_reduce(s.data_ptr(), r.data_ptr(), 7, n, 0, st.cuda_stream) == 0
    torch.cuda.synchronize()
    r.zero_()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    assert torch.all(r == 20.0)


def test_separate_allocations_capped_launch_eager_and_graph(dccl):
    """Operands of >= 512 MiB in two allocations take the aligned launch under a 22-wave cap (the shifted one under
    a 26-wave cap), chosen from a
    hipMemGetAddressRange lookup of both operands on every call (local_reduce.hip, pair_occupancy_lds).  The
    lookup must neither disturb a HIP-graph capture nor leave an error behind: eager, captured and replayed
    results are checked exactly (integer Sum), and torch's error state stays clean."""
    n = (1 << 30) // 4 + 7
    s = torch.full((n,), 3, dtype=torch.int32, device="cuda")
    r = torch.full((n,), 5, dtype=torch.int32, device="cuda")
    assert dccl.local_reduce(s.data_ptr(), r.data_ptr(), 2, n, 0, torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    assert int(r[0]) == 8 and int(r[-1]) == 8 and bool(torch.all(r == 8))
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=st):
            assert dccl.local_reduce(s.data_ptr(), r.data_ptr(), 2, n, 0, st.cuda_stream) == 0
    torch.cuda.synchronize()
    assert bool(torch.all(r == 8))  # capture does not execute
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    assert bool(torch.all(r == 14))
    del g
    # the shifted kernel (send at another 16-B phase) takes its own cap in two allocations: send 4 B further
    r.fill_(5)
    assert dccl.local_reduce(s.data_ptr() + 4, r.data_ptr(), 2, n - 1, 0, torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    assert bool(torch.all(r[:n - 1] == 8)) and int(r[n - 1]) == 5
    # the pooled layout (one allocation) of the same size runs uncapped, same result
    pool = torch.full((2 * n + 1024,), 5, dtype=torch.int32, device="cuda")
    pool[n + 1024:] = 3
    assert dccl.local_reduce(pool.data_ptr() + (n + 1024) * 4, pool.data_ptr(), 2, n, 0,
                             torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    assert bool(torch.all(pool[:n] == 8)) and bool(torch.all(pool[n:n + 1024] == 5))


def test_graph_capture_every_kernel_family(dccl):
    """Every launch path enqueues kernels only (no allocation, no host synchronisation), so each can be
    captured in one HIP graph and replayed: the pairwise combine with send off phase (shifted kernel) and
    with recv off its elements (unaligned kernel, wave-capped launch), the k-way combine with sources in
    phase, off phase (phased kernels, both forms) and at byte offsets into a misaligned recv, and the chain.
    Integer Sum, so r after R replays is exactly r0 + R * (sum of the sources) per capture."""
    n = (1 << 18) + 5
    rng = np.random.default_rng(77)
    st = torch.cuda.Stream()

    def buf(vals, off):
        t = torch.zeros(n * 4 + 64, dtype=torch.uint8, device="cuda")
        t[off:off + n * 4].copy_(torch.from_numpy(vals.view(np.uint8).copy()))
        return t, t.data_ptr() + off

    srcs = [rng.integers(-1000, 1000, n, dtype=np.int32) for _ in range(8)]
    cases = [("shift", [4], 0), ("unaligned", [0], 1), ("kway_inphase", [0, 0, 0], 0),
             ("kway_phased_small", [4, 8, 12], 0), ("kway_phased_first", [4] * 5, 0),
             ("kway_bytes", [1, 2, 3, 5], 2), ("chain", [4] * 7, 0)]
    for name, soffs, roff in cases:
        hold = [buf(srcs[j], o) for j, o in enumerate(soffs)]
        r0 = rng.integers(-1000, 1000, n, dtype=np.int32)
        tr, pr = buf(r0, roff)
        ptrs = [h[1] for h in hold]
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(st):
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=st):
                if name in ("shift", "unaligned"):
                    assert dccl.local_reduce(ptrs[0], pr, 2, n, 0, st.cuda_stream) == 0
                elif name == "chain":  # in place: dst = own + (s6 + ... + s0)
                    assert dccl.local_reduce_chain(ptrs, pr, pr, 2, n, 0, st.cuda_stream) == 0
                else:
                    assert dccl.local_reduce_multi(ptrs, pr, 2, n, 0, st.cuda_stream) == 0
        torch.cuda.synchronize()
        tr[roff:roff + n * 4].copy_(torch.from_numpy(r0.view(np.uint8).copy()))  # capture does not execute
        torch.cuda.synchronize()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        total = np.zeros(n, dtype=np.int64)
        for j in range(len(soffs)):
            total += srcs[j]
        want = (r0.astype(np.int64) + 3 * total).astype(np.int32)
        got = tr[roff:roff + n * 4].cpu().numpy().view(np.int32)
        assert np.array_equal(got, want), name
        del g
