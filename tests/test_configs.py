"""BASELINE configs C2 and C5 at their full sizes, and the line-straddling k-way / chain dispatch, on the GPU.

C2  1 x MI355X in-place two-buffer combine, ncclSum fp32, 256 MiB per operand, in both operand layouts
    (bench.py's pooled layout and DCCL's own: separately allocated scratchpad + user chunk), the whole
    result bit-exact against the oracle.
C5  one 16 GiB-per-operand fp32 Sum buffer split into 1, 2, 4 and 8 contiguous 256-B aligned shards
    (dccl_amd/shard.py, the reference's count/W slot partition, reduce_scatter_ring.cpp:22,64-65), each
    shard combined by its own dccl_local_reduce launch.  With 8 shards every shard is compared slice by
    slice, all 16 GiB, with oracle.synth + oracle.expected_reduce (as tests/test_synth.py checks C3);
    the 1-, 2- and 4-shard results must then equal the 8-shard result bit for bit on the device, and
    each of their shard boundaries is also compared with the oracle directly.
Beyond one grid  17 GiB per operand (more tiles than the 2^24-block grid cap, so every kernel's grid-stride
    loop runs): the aligned, shifted and misaligned-recv combines, the whole result checked on the device
    against the synthetic inputs regenerated per 1 GiB slice.
Straddle  in-phase k-way and chain sources off the destination's 128-B line grid (multi_straddle_typed,
    chain_straddle_typed; advisor r1): sources at 16-B multiples that are not 128-B multiples, the
    destination at another line offset, odd counts, k = 1..8, every dtype, against the sequential and
    chain-order oracle.
"""
import concurrent.futures as cf

import numpy as np
import pytest

import oracle
from dccl_amd.shard import all_bounds
from tests.test_direct import chain_expected
from tests.test_gpu_parity import dev_bytes, host_of, rand_inputs
from tests.test_oracle import fp_equal

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

SEED = 0xDCC1
GIB = 1 << 30


def _check_slices(recv_u8, lo, hi, dt=7, op=0, send_id=0, recv_id=1, piece=GIB // 4, workers=8):
    """recv elements [lo, hi) (fp32) against the oracle, in pieces of `piece` elements on a thread pool
    (the oracle's C calls release the GIL).  Returns the first mismatching piece or None."""
    def one(a):
        b = min(hi, a + piece)
        got = recv_u8[4 * a:4 * b].cpu().numpy().view(np.float32)
        s = oracle.synth(b - a, dt, op, SEED, send_id, a)
        want = oracle.synth(b - a, dt, op, SEED, recv_id, a)
        assert oracle.expected_reduce(s, want, dt, op) == 0
        return None if np.array_equal(got.view(np.uint32), want.view(np.uint32)) else (a, b)

    with cf.ThreadPoolExecutor(workers) as ex:
        bad = [x for x in ex.map(one, range(lo, hi, piece)) if x is not None]
    return bad[0] if bad else None


@pytest.mark.slow
@pytest.mark.parametrize("layout", ["pooled", "separate"])
def test_c2_256mib_against_oracle(gpu, layout):
    import dccl_amd
    nbytes = 256 << 20
    n = nbytes // 4
    if layout == "pooled":  # bench.py's layout: recv, then send 4 KiB past its end
        pool = torch.empty(2 * nbytes + 4096, dtype=torch.uint8, device="cuda")
        recv, send = pool[:nbytes], pool[nbytes + 4096:]
    else:
        send = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        recv = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    assert dccl_amd.synth_fill(send.data_ptr(), 7, n, 0, SEED, 0) == 0
    assert dccl_amd.synth_fill(recv.data_ptr(), 7, n, 0, SEED, 1) == 0
    assert dccl_amd.local_reduce(send.data_ptr(), recv.data_ptr(), 7, n, 0) == 0
    torch.cuda.synchronize()
    assert _check_slices(recv, 0, n, piece=n // 4, workers=4) is None


@pytest.mark.slow
def test_c5_16gib_sharded_against_oracle(gpu):
    import dccl_amd
    total = 16 * GIB // 4
    send = torch.empty(16 * GIB, dtype=torch.uint8, device="cuda")
    recv = torch.empty(16 * GIB, dtype=torch.uint8, device="cuda")
    assert dccl_amd.synth_fill(send.data_ptr(), 7, total, 0, SEED, 0) == 0
    ps, pr = send.data_ptr(), recv.data_ptr()
    ref = None
    for shards in (8, 4, 2, 1):
        assert dccl_amd.synth_fill(pr, 7, total, 0, SEED, 1) == 0
        bounds = all_bounds(total, 4, shards)
        for a, b in bounds:  # one launch per shard, as each GPU of the C5 config runs its own
            assert dccl_amd.local_reduce(ps + 4 * a, pr + 4 * a, 7, b - a, 0) == 0
        torch.cuda.synchronize()
        if ref is None:
            for a, b in bounds:  # every shard, slice by slice
                assert _check_slices(recv, a, b) is None, (shards, a, b)
            ref = recv.clone()
        else:
            assert torch.equal(recv, ref), shards
            for a, _ in bounds[1:]:  # both sides of every shard boundary against the oracle directly
                assert _check_slices(recv, a - 4096, a + 4096, piece=8192, workers=1) is None, (shards, a)
    del ref, recv, send
    torch.cuda.empty_cache()


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 6, 7, 8])
def test_kway_and_chain_line_straddling_sources(gpu, k):
    import dccl_amd
    rng = np.random.default_rng(700 + k)
    for dt in range(10):
        esz = int(oracle.NP_DTYPES[dt]().itemsize)
        for n in (1, 3, 63, 4099, 65537):
            op = int(rng.integers(0, 4))
            sends = [rand_inputs(rng, dt, n)[0] for _ in range(k)]
            _, r = rand_inputs(rng, dt, n)
            soffs = [int(rng.choice([16, 48, 80, 112, 144, 208])) for _ in range(k)]
            roff = int(rng.choice([0, 32, 64, 96]))
            holders = [dev_bytes(x, o) for x, o in zip(sends, soffs)]
            # k-way: recv = op(...op(recv, s0)..., s{k-1})
            tr, pr = dev_bytes(r, roff)
            assert dccl_amd.local_reduce_multi([h[1] for h in holders], pr, dt, n, op, 0) == 0
            torch.cuda.synchronize()
            want = r
            for x in sends:
                want = oracle.combine(x, want, dt, op)
            assert fp_equal(host_of(tr, roff, r), want, dt), ("multi", k, dt, n, op, soffs, roff)
            # chain, in place (own == dst) and into a separate dst at another line offset
            want_c = chain_expected(sends, r, dt, op)
            to, po = dev_bytes(r, roff)
            assert dccl_amd.local_reduce_chain([h[1] for h in holders], po, po, dt, n, op, 0) == 0
            doff = (roff + 64) % 128
            td, pd = dev_bytes(np.zeros_like(r), doff)
            to2, po2 = dev_bytes(r, doff)
            assert dccl_amd.local_reduce_chain([h[1] for h in holders], po2, pd, dt, n, op, 0) == 0
            torch.cuda.synchronize()
            assert fp_equal(host_of(to, roff, r), want_c, dt), ("chain", k, dt, n, op, soffs, roff)
            assert fp_equal(host_of(td, doff, r), want_c, dt), ("chain dst", k, dt, n, op, soffs, doff)
            assert host_of(to2, doff, r).tobytes() == r.tobytes()  # own untouched


@pytest.mark.slow
@pytest.mark.parametrize("dt,roff,soff", [(7, 1, 0), (7, 2, 7), (8, 3, 0), (8, 4, 12), (9, 1, 0), (2, 3, 2)])
def test_recv_misaligned_large_against_oracle(gpu, dt, roff, soff):
    """A recv that is not element-aligned (reduce_unaligned_kernel: one 16-B access per lane at
    the displaced addresses) at 64 MiB, across
    many tiles and grid strides: the whole result against the oracle, nothing outside recv written."""
    import dccl_amd
    esz = int(oracle.NP_DTYPES[dt]().itemsize)
    n = (64 << 20) // esz + 5
    op = 0 if dt != 9 else 2
    s = oracle.synth(n, dt, op, SEED, 40)
    r = oracle.synth(n, dt, op, SEED, 41)
    ts, ps = dev_bytes(s, soff)
    tr, pr = dev_bytes(r, roff)
    assert dccl_amd.local_reduce(ps, pr, dt, n, op, 0) == 0
    torch.cuda.synchronize()
    got = host_of(tr, roff, r)
    assert got.tobytes() == oracle.combine(s, r, dt, op).tobytes()
    nb = n * esz
    assert not tr[:roff].any() and not tr[roff + nb:].any()


@pytest.mark.slow
@pytest.mark.parametrize("soff,roff", [(0, 0), (4, 0), (0, 1)], ids=["aligned", "send_phase4", "recv_plus1"])
def test_beyond_max_grid_17gib(gpu, soff, roff):
    """fp32 Sum over 17 GiB per operand: 2^24 one-wave blocks cover 16 GiB, so the grid-stride loop of the
    vector kernel (aligned), the shifted kernel (send 4 B off phase) and reduce_unaligned_kernel (recv 1 B
    off) all run a second pass.  Operands are written slice by slice from the counter-based generator
    (dccl_synth_fill_range into an aligned slice, then a byte copy to the operand's offset); the result is
    compared bit for bit with recv + send recomputed by torch per 1 GiB slice; the bytes around recv stay."""
    import dccl_amd
    total = 17 * (GIB // 4)
    piece = GIB // 4
    nb = 4 * total
    send = torch.zeros(nb + 4096, dtype=torch.uint8, device="cuda")
    recv = torch.zeros(nb + 4096, dtype=torch.uint8, device="cuda")
    a = torch.empty(piece, dtype=torch.float32, device="cuda")
    b = torch.empty(piece, dtype=torch.float32, device="cuda")
    for first in range(0, total, piece):
        m = min(piece, total - first)
        assert dccl_amd.synth_fill_range(a.data_ptr(), 7, m, 0, SEED, 60, first) == 0
        assert dccl_amd.synth_fill_range(b.data_ptr(), 7, m, 0, SEED, 61, first) == 0
        send[soff + 4 * first:soff + 4 * (first + m)].copy_(a[:m].view(torch.uint8))
        recv[roff + 4 * first:roff + 4 * (first + m)].copy_(b[:m].view(torch.uint8))
    assert dccl_amd.local_reduce(send.data_ptr() + soff, recv.data_ptr() + roff, 7, total, 0) == 0
    torch.cuda.synchronize()
    got = torch.empty(piece, dtype=torch.float32, device="cuda")
    for first in range(0, total, piece):
        m = min(piece, total - first)
        assert dccl_amd.synth_fill_range(a.data_ptr(), 7, m, 0, SEED, 60, first) == 0
        assert dccl_amd.synth_fill_range(b.data_ptr(), 7, m, 0, SEED, 61, first) == 0
        got[:m].view(torch.uint8).copy_(recv[roff + 4 * first:roff + 4 * (first + m)])
        want = b[:m] + a[:m]
        assert torch.equal(got[:m].view(torch.int32), want.view(torch.int32)), (soff, roff, first)
    assert not recv[:roff].any() and not recv[roff + nb:].any()
    del send, recv, a, b, got
    torch.cuda.empty_cache()


@pytest.mark.slow
@pytest.mark.parametrize("kind,soff,roff", [("multi", 0, 0), ("multi", 4, 0), ("multi", 0, 2), ("chain", 0, 0),
                                            ("chain", 4, 0), ("chain", 0, 2)])
def test_kway_chain_beyond_max_grid_17gib(gpu, kind, soff, roff):
    """The k-way (k = 2) and chain (k = 2, separate dst) combines over 17 GiB per operand, past the grid cap:
    in phase (vector kernels), sources 4 B off phase (phased kernels), destination 2 B off (unaligned
    kernels).  Checked bit for bit per 1 GiB slice against torch on the regenerated inputs, in the
    kernels' association order (k-way: (recv + s0) + s1; chain: own + (s1 + s0))."""
    import dccl_amd
    total = 17 * (GIB // 4)
    piece = GIB // 4
    nb = 4 * total
    bufs = [torch.zeros(nb + 4096, dtype=torch.uint8, device="cuda") for _ in range(3)]  # s0, s1, recv / own
    dst = torch.zeros(nb + 4096, dtype=torch.uint8, device="cuda") if kind == "chain" else None
    offs = [soff, soff, roff if kind == "multi" else 0]
    tmp = torch.empty(piece, dtype=torch.float32, device="cuda")
    for first in range(0, total, piece):
        m = min(piece, total - first)
        for j, (buf, off) in enumerate(zip(bufs, offs)):
            assert dccl_amd.synth_fill_range(tmp.data_ptr(), 7, m, 0, SEED, 70 + j, first) == 0
            buf[off + 4 * first:off + 4 * (first + m)].copy_(tmp[:m].view(torch.uint8))
    ptrs = [b.data_ptr() + o for b, o in zip(bufs, offs)]
    if kind == "multi":
        assert dccl_amd.local_reduce_multi(ptrs[:2], ptrs[2], 7, total, 0, 0) == 0
        out, ooff = bufs[2], roff
    else:
        assert dccl_amd.local_reduce_chain(ptrs[:2], ptrs[2], dst.data_ptr() + roff, 7, total, 0) == 0
        out, ooff = dst, roff
    torch.cuda.synchronize()
    v = [torch.empty(piece, dtype=torch.float32, device="cuda") for _ in range(3)]
    for first in range(0, total, piece):
        m = min(piece, total - first)
        for j in range(3):
            assert dccl_amd.synth_fill_range(v[j].data_ptr(), 7, m, 0, SEED, 70 + j, first) == 0
        want = (v[2][:m] + v[0][:m]) + v[1][:m] if kind == "multi" else v[2][:m] + (v[1][:m] + v[0][:m])
        tmp[:m].view(torch.uint8).copy_(out[ooff + 4 * first:ooff + 4 * (first + m)])
        assert torch.equal(tmp[:m].view(torch.int32), want.view(torch.int32)), (kind, soff, roff, first)
    assert not out[:ooff].any() and not out[ooff + nb:].any()
    del bufs, dst, tmp, v, out
    torch.cuda.empty_cache()


@pytest.mark.slow
def test_host_staged_count_beyond_2_32(gpu):
    """Host-resident operands (DCCL's RDMA buffers) with more than 2^32 elements: int8 Sum over 4.5 GiB of
    pageable memory through the host-staged path (the reference caps its host scratchpad at 4 GiB and keeps
    slice sizes in uint32), checked slice by slice against the oracle."""
    import dccl_amd
    n = 4 * GIB + GIB // 2  # int8: elements == bytes > 2^32
    s = oracle.synth(n, 0, 0, SEED, 80)
    r = oracle.synth(n, 0, 0, SEED, 81)
    assert dccl_amd.local_reduce_host(s.ctypes.data, r.ctypes.data, 0, n, 0) == 0
    piece = GIB // 4

    def one(a):
        b = min(n, a + piece)
        want = oracle.synth(b - a, 0, 0, SEED, 81, a)
        assert oracle.expected_reduce(s[a:b], want, 0, 0) == 0
        return None if np.array_equal(r[a:b], want) else (a, b)

    with cf.ThreadPoolExecutor(8) as ex:
        bad = [x for x in ex.map(one, range(0, n, piece)) if x is not None]
    assert not bad, bad[:3]
    assert np.array_equal(s[-4096:], oracle.synth(4096, 0, 0, SEED, 80, n - 4096))  # send untouched
