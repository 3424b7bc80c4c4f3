"""The script that made the committed golden fixtures for the local combine.

    make -C oracle && python tests/golden/make_golden.py      (regenerates host_reduce_half.npz)

Outputs (data only: inputs and expected outputs):

* ``host_reduce_ref.npz`` — for every host dtype the reference supports
  (int8, uint8, int32, uint32, int64, uint64, float32, float64) x sizes
  {1, 15, 16, 17, 255, 256, 1000, 4099}: seeded ``send`` / ``recv`` inputs (special values
  spliced in) and, per op {Sum, Prod, Max, Min}, the output of the reference's
  ``do_host_reduce<DT>`` (/root/reference/src/core/internal_common.hpp:496-586) as built in round 1.
  FROZEN: that build stood in for the reference's CMake-generated config.h and for spdlog, which the
  rules count as unbuildable, so it was removed in round 2 and these files are regression data for the
  restatement, not a pin of it (parity unpinned).  ``gen_ref``, ``gen_misaligned`` and
  ``gen_rc`` are kept as the record of how they were made; they need that removed build
  (``_ref_reduce`` below) and no longer run.
* ``host_reduce_half.npz`` — float16 / bfloat16 (no reference host path: SURVEY.md
  A.2/A.3 #6): outputs of numpy float16 arithmetic and torch CPU bfloat16 arithmetic
  — independent of both the oracle and the HIP kernel.
* ``misaligned_ref.npz`` — SURVEY.md A.4 cases (recv off a 64-B line): the reference's output
  (it re-combines the tail and writes past `count`) next to the correct result the build gives.
* ``rc_cases.json`` — return codes of the reference for Avg / bad op / count 0.

The C1 ring goldens (dccl_cli all_reduce) live in ``c1_ring.json``,
whose values are the bit patterns captured from the reference by the survey and
re-derived here by simulating the reference ring choreography around the compiled
reference combine.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import oracle  # noqa: E402  (test infrastructure)

SIZES = [1, 15, 16, 17, 255, 256, 1000, 4099]
HOST_DTYPES = [0, 1, 2, 3, 4, 5, 7, 8]
OPS = [0, 1, 2, 3]
SEED = 0xDCC1


def special_values(npd) -> np.ndarray:
    if np.issubdtype(npd, np.integer):
        info = np.iinfo(npd)
        return np.array([info.min, info.max, 0, 1, info.max, info.min, 100, -1 if info.min < 0 else 200],
                        dtype=npd)
    f = np.finfo(npd)
    return np.array([np.nan, 1.0, 0.0, -0.0, np.inf, -np.inf, f.tiny / 4, -f.tiny / 2, f.max, 2.0],
                    dtype=npd)


def special_partners(npd) -> np.ndarray:
    if np.issubdtype(npd, np.integer):
        info = np.iinfo(npd)
        return np.array([info.min, 1, info.max, info.max, info.max, -1 if info.min < 0 else 255, 100,
                         3], dtype=npd)
    f = np.finfo(npd)
    return np.array([1.0, np.nan, -0.0, 0.0, -np.inf, 1.0, f.tiny / 4, f.tiny, f.max, np.nan], dtype=npd)


def make_inputs(rng, npd, n):
    if np.issubdtype(npd, np.integer):
        info = np.iinfo(npd)
        s = rng.integers(info.min, info.max, n, dtype=npd, endpoint=True)
        r = rng.integers(info.min, info.max, n, dtype=npd, endpoint=True)
    else:
        s = rng.uniform(-1, 1, n).astype(npd)
        r = rng.uniform(-1, 1, n).astype(npd)
    k = min(n, len(special_values(npd)))
    if n >= 8:  # splice specials at the start (recv, send) and mirrored (send, recv) at the end
        r[:k] = special_values(npd)[:k]
        s[:k] = special_partners(npd)[:k]
        r[n - k:] = special_partners(npd)[:k]
        s[n - k:] = special_values(npd)[:k]
    return s, r


def _ref_reduce(*args, **kw):
    raise SystemExit("the round-1 reference build (oracle/_ref) was removed: the *_ref fixtures are frozen")


def aligned_copy(a: np.ndarray) -> np.ndarray:
    b = oracle.aligned_empty(a.size, a.dtype)
    b[:] = a
    return b


def gen_ref():
    rng = np.random.default_rng(SEED)
    out = {}
    for dt in HOST_DTYPES:
        npd = oracle.NP_DTYPES[dt]
        for n in SIZES:
            s, r = make_inputs(rng, npd, n)
            out[f"d{dt}_n{n}_send"] = s
            out[f"d{dt}_n{n}_recv"] = r
            for op in OPS:
                rr = aligned_copy(r)
                rc = _ref_reduce(aligned_copy(s), rr, dt, op)
                assert rc == 0, (dt, n, op, rc)
                out[f"d{dt}_n{n}_op{op}_out"] = np.array(rr)
    np.savez_compressed(os.path.join(HERE, "host_reduce_ref.npz"), **out)


def gen_half():
    import torch

    rng = np.random.default_rng(SEED + 1)
    out = {}
    for dt, name in ((6, "f16"), (9, "bf16")):
        for n in SIZES:
            s = rng.uniform(-2, 2, n).astype(np.float32)
            r = rng.uniform(-2, 2, n).astype(np.float32)
            if n >= 8:
                r[:8] = [np.nan, 1.0, 0.0, -0.0, np.inf, 65504.0, 6e-8, 3e38]
                s[:8] = [1.0, np.nan, -0.0, 0.0, -np.inf, 65504.0, 6e-8, 3e38]
            if dt == 6:
                s16, r16 = s.astype(np.float16), r.astype(np.float16)
                sb, rb = s16.view(np.uint16), r16.view(np.uint16)
                outs = [(r16 + s16), (r16 * s16), np.where(r16 < s16, s16, r16), np.where(r16 > s16, s16, r16)]
                outs = [o.astype(np.float16).view(np.uint16) for o in outs]
            else:
                st, rt = torch.from_numpy(s).bfloat16(), torch.from_numpy(r).bfloat16()
                sb = st.view(torch.int16).numpy().view(np.uint16)
                rb = rt.view(torch.int16).numpy().view(np.uint16)
                outs = [rt + st, rt * st, torch.where(rt < st, st, rt), torch.where(rt > st, st, rt)]
                outs = [o.view(torch.int16).numpy().view(np.uint16) for o in outs]
            out[f"d{dt}_n{n}_send"] = sb.copy()
            out[f"d{dt}_n{n}_recv"] = rb.copy()
            for op, o in zip(OPS, outs):
                out[f"d{dt}_n{n}_op{op}_out"] = o.copy()
    np.savez_compressed(os.path.join(HERE, "host_reduce_half.npz"), **out)


def gen_misaligned():
    """SURVEY.md A.4 'reference-wrong, build-correct' expectations: recv off a 64-B line with
    count % P < head.  The reference loop (run on padded buffers) re-combines the tail and writes
    past `count`; the build must produce the plain element-wise result."""
    rng = np.random.default_rng(SEED + 2)
    out = {}
    cases = [(7, 32, 100), (7, 4, 33), (2, 48, 70), (8, 8, 13), (0, 1, 130), (4, 16, 21)]
    for i, (dt, off, n) in enumerate(cases):
        npd = oracle.NP_DTYPES[dt]
        pad = 64
        if np.issubdtype(npd, np.integer):
            info = np.iinfo(npd)
            s = rng.integers(info.min // 2, info.max // 2, n + pad, dtype=npd)
            r = rng.integers(info.min // 2, info.max // 2, n + pad, dtype=npd)
        else:
            s = rng.uniform(-1, 1, n + pad).astype(npd)
            r = rng.uniform(-1, 1, n + pad).astype(npd)
        ss = oracle.aligned_empty(n + pad, npd, offset_bytes=off)
        rr = oracle.aligned_empty(n + pad, npd, offset_bytes=off)
        ss[:] = s
        rr[:] = r
        assert _ref_reduce(ss, rr, dt, 0, count=n) == 0  # Sum over the first n only
        correct = r.copy()
        correct[:n] = oracle.combine(s[:n], r[:n], dt, 0)
        out[f"c{i}_meta"] = np.array([dt, off, n], dtype=np.int64)
        out[f"c{i}_send"] = s
        out[f"c{i}_recv"] = r
        out[f"c{i}_ref"] = np.array(rr)        # reference result incl. the overrun into the padding
        out[f"c{i}_correct"] = correct         # build contract: only [0, n) changes
    np.savez_compressed(os.path.join(HERE, "misaligned_ref.npz"), **out)


def gen_rc():
    cases = []
    for dt in HOST_DTYPES:
        npd = oracle.NP_DTYPES[dt]
        for op in (4, 5, 7):
            for n in (0, 16):
                s = oracle.aligned_empty(max(n, 1), npd)
                r = oracle.aligned_empty(max(n, 1), npd)
                rc = _ref_reduce(s, r, dt, op, count=n)
                cases.append({"dtype": dt, "op": op, "count": n, "rc": rc})
    with open(os.path.join(HERE, "rc_cases.json"), "w") as f:
        json.dump(cases, f, indent=0)


if __name__ == "__main__":
    gen_half()  # gen_ref / gen_misaligned / gen_rc: frozen (see the module docstring)
    print("golden fixtures written to", HERE)
