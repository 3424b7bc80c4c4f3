"""The resident-wave caps of the capped combine launches (dccl_amd/csrc/caps.hpp), on the CPU: caps.hpp is
host-only C++, compiled here with g++ into a small harness that prints caps::waves / caps::lds for every
(kernel class, k) the launchers can ask for.  Every cap is a legal LDS request (<= 64 KiB per block), k outside
[1, 8] (or a class's own range) is rejected, and the table is the frozen one below — changing an entry means
changing this test, with the measurement that justifies it (>= 2 points, two boxes)."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "dccl_amd", "csrc")

HARNESS = r"""
#include <cstdio>
#include "caps.hpp"
using namespace dccl_amd::caps;
int main() {
    const size_t MiB = size_t(1) << 20;
    const size_t sizes[] = {4096, 24 * MiB - 1, 24 * MiB, 48 * MiB - 1, 48 * MiB, 96 * MiB - 1, 96 * MiB, 1024 * MiB};
    std::printf("{\"rows\": [");
    bool first = true;
    for (int c = 0; c < kNumKernels; ++c)
        for (size_t b : sizes)
            for (int k = -1; k <= 9; ++k) {
                std::printf("%s[%d, %zu, %d, %d, %zu]", first ? "" : ", ", c, b, k, waves(Kernel(c), k, b),
                            lds(Kernel(c), k, b));
                first = false;
            }
    std::printf("], \"runs\": [");
    for (int c = 0; c < kNumKernels; ++c)
        for (int k = 0; k <= 8; ++k) std::printf("%s%d", (c || k) ? ", " : "", tile_run(Kernel(c), k));
    std::printf("], \"loads_first\": [");
    for (int ch = 0; ch < 2; ++ch)
        for (int k = 1; k <= 8; ++k) std::printf("%s%d", (ch || k > 1) ? ", " : "", int(phased_loads_first(ch, k)));
    std::printf("], \"windows\": [");
    for (int c = 0; c < kNumWindowClasses; ++c)
        for (int k = 0; k <= 8; ++k) {
            const WindowForm f = window_form(WindowClass(c), k);
            std::printf("%s[%d, %d, %d, %d, %zu]", (c || k) ? ", " : "", c, k, f.first * 100 + f.order * 10, f.waves,
                        lds_for_waves(f.waves));
        }
    std::printf("], \"window_mid\": [");
    const size_t mids[] = {kWindowMidBytes - 1, kWindowMidBytes, kWindowTunedBytes - 1, kWindowTunedBytes};
    for (int ch = 0; ch < 2; ++ch)
        for (int k = 1; k <= 8; ++k)
            for (size_t b : mids)
                std::printf("%s[%d, %d, %zu, %d, %d, %d]", (ch || k > 1 || b != mids[0]) ? ", " : "", ch, k, b,
                            int(window_mid(ch, k, b)), int(phased_via_windows(ch, k, b, true)),
                            int(phased_via_windows(ch, k, b, false)));
    std::printf("], \"mid_forms\": [%d, %d]}\n", kWindowMid.first * 1000 + kWindowMid.order * 100 + kWindowMid.waves,
                kWindowMidChain3.first * 1000 + kWindowMidChain3.order * 100 + kWindowMidChain3.waves);
}
"""

NAMES = ["multi", "chain", "multi_straddle", "chain_straddle", "multi_phased_first", "chain_phased_first"]
# frozen table: class -> size class (<24, <48, <96 MiB, >=96 MiB) -> waves for k = 0..8 (0 = not used at that k;
# for the phased classes 0 = the per-operand form)
FROZEN = {
    "multi": [[0, 0, 32, 24, 16, 16, 16, 10, 9], [0, 0, 32, 20, 13, 11, 11, 10, 9],
              [0, 0, 24, 16, 13, 11, 11, 10, 9], [0, 0, 18, 13, 13, 11, 11, 10, 9]],
    "chain": [[0, 32, 32, 32, 16, 24, 16, 16, 16], [0, 32, 32, 32, 16, 16, 16, 16, 9],
              [0, 32, 32, 20, 16, 13, 11, 10, 9], [0, 32, 24, 20, 16, 13, 11, 10, 9]],
    "multi_straddle": [[0, 0, 32, 24, 16, 16, 16, 9, 9], [0, 0, 24, 16, 13, 11, 9, 9, 9],
                       [0, 0, 24, 16, 13, 11, 9, 9, 9], [0, 0, 18, 13, 13, 11, 9, 9, 9]],
    "chain_straddle": [[0, 32, 24, 32, 24, 24, 16, 10, 9], [0, 32, 32, 32, 24, 13, 11, 10, 9],
                       [0, 32, 32, 24, 16, 13, 11, 10, 9], [0, 32, 24, 18, 13, 13, 11, 10, 9]],
    "multi_phased_first": [[0, 0, 0, 0, 16, 16, 13, 24, 13], [0, 0, 0, 0, 16, 16, 13, 13, 13],
                           [0, 0, 0, 0, 16, 13, 13, 13, 13], [0, 0, 0, 0, 16, 13, 13, 13, 13]],
    "chain_phased_first": [[0, 0, 0, 16, 24, 24, 0, 24, 16], [0, 0, 0, 16, 16, 16, 0, 13, 24],
                           [0, 0, 0, 16, 13, 13, 0, 13, 11], [0, 0, 0, 16, 13, 13, 0, 13, 11]],
}
K_RANGE = {"multi": (2, 8), "chain": (1, 8), "multi_straddle": (2, 8), "chain_straddle": (1, 8),
           "multi_phased_first": (2, 8), "chain_phased_first": (1, 8)}


@pytest.fixture(scope="module")
def table(tmp_path_factory):
    d = tmp_path_factory.mktemp("caps")
    src, exe = d / "caps_dump.cpp", d / "caps_dump"
    src.write_text(HARNESS)
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", f"-I{CSRC}", str(src), "-o", str(exe)],
                   check=True)
    return json.loads(subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout)


def size_class(b):
    return 0 if b < 24 << 20 else 1 if b < 48 << 20 else 2 if b < 96 << 20 else 3


def lds_for(w):
    return 0 if w <= 0 or w >= 32 else ((160 << 10) // w + 255) // 256 * 256


def test_every_entry_is_the_frozen_table_and_a_legal_request(table):
    seen = 0
    for c, b, k, w, lds in table["rows"]:
        name = NAMES[c]
        lo, hi = K_RANGE[name]
        if not lo <= k <= hi:
            assert w == -1 and lds == 0, (name, k)  # k outside the class's range: rejected, no request
            continue
        assert w == FROZEN[name][size_class(b)][k], (name, b, k, w)
        assert lds == lds_for(w) and lds <= 64 << 10, (name, b, k, lds)
        if w:
            assert 7 <= w <= 32 and (lds == 0) == (w == 32)
            assert (160 << 10) // lds >= w - 2 if lds else True  # the request really caps near w waves
        seen += 1
    assert seen == sum(8 * (hi - lo + 1) for lo, hi in K_RANGE.values())


def test_size_class_boundaries(table):
    rows = {(NAMES[c], b, k): w for c, b, k, w, _ in table["rows"]}
    MiB = 1 << 20
    # kMulti k = 3 switches 24 -> 20 -> 16 -> 13 at 24 / 48 / 96 MiB
    assert [rows[("multi", b, 3)] for b in (24 * MiB - 1, 24 * MiB, 48 * MiB - 1, 48 * MiB, 96 * MiB - 1, 96 * MiB)] \
        == [24, 20, 20, 16, 16, 13]
    assert rows[("multi", 1024 * MiB, 8)] == rows[("multi", 96 * MiB, 8)] == 9


def test_phased_form_is_fixed_per_k(table):
    lf = table["loads_first"]
    assert lf[:8] == [0, 0, 0, 1, 1, 1, 1, 1]   # k-way: loads-first from k = 4
    assert lf[8:] == [0, 0, 1, 1, 1, 0, 1, 1]   # chain: at k = 3, 4, 5, 7, 8


def test_tile_runs(table):
    runs = table["runs"]
    want = {"multi_straddle": {8: 4}, "multi_phased_first": {4: 4, 6: 4, 7: 4, 8: 4},
            "chain_phased_first": {3: 4, 7: 4, 8: 4}}
    for c, name in enumerate(NAMES):
        for k in range(9):
            assert runs[9 * c + k] == want.get(name, {}).get(k, 1), (name, k)


def test_window_forms(table):
    """reduce_windows_kernel's tuned forms (caps.hpp kWindow): per-operand block order under 26
    waves in phase from k = 3; off phase per-operand in group order at k = 3 (26), loads-first in group order at
    k = 4 (14 waves) and 5 (12), loads-first in runs of 4 at k = 6..8 (13); k <= 2 uncapped; the phased launches
    at k-way k = 3..5 and chain k = 4..7 from 96 MiB per operand."""
    want = {0: {k: (10, 26 if k >= 3 else 32) for k in range(9)},
            1: {k: (0, 32) if k <= 2 else (20, 26) if k == 3 else (120, 14) if k == 4 else (120, 12) if k == 5
                else (130, 13) for k in range(9)}}
    for c, k, form, w, lds in table["windows"]:
        assert (form, w) == want[c][k], (c, k, form, w)
        assert lds == lds_for(w) and lds <= 64 << 10


def test_window_mid_sizes(table):
    """From 48 to 96 MiB per operand (caps.hpp window_mid): with sources off phase, k = 4..8 take the loads-first
    tile in group order under 14 waves and the chain at k = 3 the per-operand tile in group order under 26;
    phased launches with the destination at 16-B phase 0 take them too.  From 96 MiB the 1 GiB table rules
    (phased routing independent of the destination's phase)."""
    assert table["mid_forms"] == [1214, 226]
    for ch, k, b, mid, via_dst16, via_not16 in table["window_mid"]:
        in_mid = (48 << 20) <= b < (96 << 20)
        assert mid == int((3 if ch else 4) <= k <= 8 and in_mid), (ch, k, b)
        if b >= 96 << 20:
            want = int((4 <= k <= 7) if ch else (3 <= k <= 5))
            assert via_dst16 == want and via_not16 == want, (ch, k, b)
        else:
            assert via_dst16 == mid and via_not16 == 0, (ch, k, b)
