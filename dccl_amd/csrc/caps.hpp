// dccl_amd/csrc/caps.hpp — resident-wave caps of every capped combine launch and the functions that select them.
// Host-only C++: tests/test_caps.py compiles it with g++ and freezes every entry; table_ok() checks it at build.
// Every combine kernel is a one-wave block streaming 16-B vectors; with k + 1 loads per lane in flight, too many
// resident waves put too many bytes in flight for the DRAM.  A launch asks for `bytes` of unused dynamic LDS per
// block, so a CU holds floor(160 KiB / bytes) of them; values are NOMINAL wave counts (the 256-B rounding makes
// 8 and 9, 16 and 18 the same occupancy).  An entry stays only if it leads the simpler choice by >= 2 points on
// two boxes (round 5 removed the straddle bands, the separate-allocation pair cap and every size-row
// cell below that bar: tools/ab_cases.py, profiles/r5_ab_caps.json).
#pragma once

#include <cstddef>

namespace dccl_amd {
namespace caps {

// Kernel classes that take a cap.  Values index kWaves.
enum Kernel : int {
    kMulti = 0,         // reduce_multi_vec_kernel, sources in phase and on recv's 128-B lines (k = 2..8)
    kChain,             // reduce_chain_vec_kernel, the same (k = 1..8)
    kMultiStraddle,     // reduce_multi_vec_kernel, in-phase sources off recv's lines (loaded through the caches)
    kChainStraddle,     // reduce_chain_vec_kernel, the same
    kMultiPhasedFirst,  // reduce_multi_phased_kernel, loads-first form; 0 = the per-operand form, uncapped
    kChainPhasedFirst,  // reduce_chain_phased_kernel, the same
    kNumKernels
};

inline constexpr int kUncapped = 32;  // 32 one-wave blocks per CU: the hardware limit
inline constexpr size_t kLdsPerCu = size_t(160) << 10;
inline constexpr size_t kMaxLdsPerBlock = size_t(64) << 10;

// Size class by bytes per operand: 0, 1, 2 below 24, 48, 96 MiB; 3 (the 1 GiB row) above (small launches: few
// tiles per resident wave, the tail dominates, more waves win).
inline constexpr int kSizeClasses = 4;
constexpr int size_class(size_t bytes) {
    return bytes < (size_t(24) << 20) ? 0 : bytes < (size_t(48) << 20) ? 1 : bytes < (size_t(96) << 20) ? 2 : 3;
}

// kWaves[kernel][size class][k]: nominal resident waves per CU (32 = uncapped; 0 = not used at that k, or for
// the phased classes the per-operand form).  1 GiB row: the best caps of rounds 1-3's sweeps; a smaller class
// keeps its own value only where it led the 1 GiB value by >= 2 points (profiles/r5_ab_caps.json).
inline constexpr unsigned char kWaves[kNumKernels][kSizeClasses][9] = {
    // k:  0  1   2   3   4   5   6   7   8
    {{0, 0, 32, 24, 16, 16, 16, 10, 9},  // kMulti            < 24 MiB
     {0, 0, 32, 20, 13, 11, 11, 10, 9},  //                   < 48 MiB
     {0, 0, 24, 16, 13, 11, 11, 10, 9},  //                   < 96 MiB
     {0, 0, 18, 13, 13, 11, 11, 10, 9}}, //                   1 GiB row
    {{0, 32, 32, 32, 16, 24, 16, 16, 16},  // kChain
     {0, 32, 32, 32, 16, 16, 16, 16, 9},
     {0, 32, 32, 20, 16, 13, 11, 10, 9},
     {0, 32, 24, 20, 16, 13, 11, 10, 9}},
    {{0, 0, 32, 24, 16, 16, 16, 9, 9},  // kMultiStraddle
     {0, 0, 24, 16, 13, 11, 9, 9, 9},
     {0, 0, 24, 16, 13, 11, 9, 9, 9},
     {0, 0, 18, 13, 13, 11, 9, 9, 9}},
    {{0, 32, 24, 32, 24, 24, 16, 10, 9},  // kChainStraddle
     {0, 32, 32, 32, 24, 13, 11, 10, 9},
     {0, 32, 32, 24, 16, 13, 11, 10, 9},
     {0, 32, 24, 18, 13, 13, 11, 10, 9}},
    {{0, 0, 0, 0, 16, 16, 13, 24, 13},  // kMultiPhasedFirst: loads-first from k = 4
     {0, 0, 0, 0, 16, 16, 13, 13, 13},
     {0, 0, 0, 0, 16, 13, 13, 13, 13},
     {0, 0, 0, 0, 16, 13, 13, 13, 13}},
    {{0, 0, 0, 16, 24, 24, 0, 24, 16},  // kChainPhasedFirst: at k = 3, 4, 5, 7, 8
     {0, 0, 0, 16, 16, 16, 0, 13, 24},
     {0, 0, 0, 16, 13, 13, 0, 13, 11},
     {0, 0, 0, 16, 13, 13, 0, 13, 11}},
};

// kRun[kernel][k]: tile-run order (run_tile<RUN>: each XCD walks RUN consecutive tiles; 1 = block order).  Runs
// of 4 keep the line two neighbouring tiles share in one L2 in 3 of 4 cases (+2.0..+3.7 points, round 3).
inline constexpr unsigned char kRun[kNumKernels][9] = {
    {1, 1, 1, 1, 1, 1, 1, 1, 1},  // kMulti
    {1, 1, 1, 1, 1, 1, 1, 1, 1},  // kChain
    {1, 1, 1, 1, 1, 1, 1, 1, 4},  // kMultiStraddle
    {1, 1, 1, 1, 1, 1, 1, 1, 1},  // kChainStraddle
    {1, 1, 1, 1, 4, 1, 4, 4, 4},  // kMultiPhasedFirst
    {1, 1, 1, 4, 1, 1, 1, 4, 4},  // kChainPhasedFirst
};
constexpr int tile_run(Kernel c, int k) { return (c < 0 || c >= kNumKernels || k < 0 || k > 8) ? 1 : kRun[c][k]; }

// The valid k range of each class (the launchers' with_k bounds).
constexpr int min_k(Kernel c) { return c == kMulti || c == kMultiStraddle || c == kMultiPhasedFirst ? 2 : 1; }
constexpr int max_k(Kernel) { return 8; }
// Nominal waves of a launch (class c, k sources, `bytes` per operand); -1 for a k outside the class's range.
constexpr int waves(Kernel c, int k, size_t bytes) {
    return (c < 0 || c >= kNumKernels || k < min_k(c) || k > max_k(c)) ? -1 : kWaves[c][size_class(bytes)][k];
}

// Dynamic LDS bytes per one-wave block for a nominal wave count (0 = no request: uncapped), and of a launch.
constexpr size_t lds_for_waves(int w) { return (w <= 0 || w >= kUncapped) ? 0 : (kLdsPerCu / size_t(w) + 255) / 256 * 256; }
constexpr size_t lds(Kernel c, int k, size_t bytes) { return lds_for_waves(waves(c, k, bytes)); }

// Does the phased k-way (chain) launch with k sources take the loads-first form?  Per K (every size row agrees).
constexpr bool phased_loads_first(bool chain, int k) {
    return waves(chain ? kChainPhasedFirst : kMultiPhasedFirst, k, size_t(1) << 30) > 0;
}

// ---- reduce_windows_kernel (k-way / chain into a destination at its own 16-B phase) ----
// From kWindowTunedBytes: per-operand tile under 26 waves (sources in phase, +2.1..+3.5 points) or, sources off
// phase, the loads-first tile under 12-14 waves (+0.5..+5.3; k = 3 per-operand, 26).  From kWindowMidBytes with
// sources off phase one mid-size form (+3..+7 over the phased kernels at 64 MiB).  Else per-operand, uncapped.
inline constexpr size_t kWindowTunedBytes = size_t(96) << 20;
inline constexpr size_t kWindowMidBytes = size_t(48) << 20;
enum WindowClass : int { kWinInPhase = 0, kWinOffPhase, kNumWindowClasses };
struct WindowForm {
    unsigned char first;  // 1: loads-first tile
    unsigned char order;  // reduce_kernels.hpp kOrderXcd (0), kOrderBlock (1), kOrderGroup (2), kOrderRun4 (3)
    unsigned char waves;  // resident-wave cap (32 = uncapped)
};
inline constexpr WindowForm kWindow[kNumWindowClasses][9] = {
    // k = 0, 1, 2: the round-3 kernels (in phase) or the uncapped XCD-range form (off phase)
    {{0, 1, 32}, {0, 1, 32}, {0, 1, 32}, {0, 1, 26}, {0, 1, 26}, {0, 1, 26}, {0, 1, 26}, {0, 1, 26}, {0, 1, 26}},
    {{0, 0, 32}, {0, 0, 32}, {0, 0, 32}, {0, 2, 26}, {1, 2, 14}, {1, 2, 12}, {1, 3, 13}, {1, 3, 13}, {1, 3, 13}},
};
constexpr WindowForm window_form(WindowClass c, int k) { return kWindow[c][k < 0 ? 0 : k > 8 ? 8 : k]; }
constexpr WindowForm kWindowMid{1, 2, 14}, kWindowMidChain3{0, 2, 26};
constexpr bool window_mid(bool chain, int k, size_t bytes) {
    return k >= (chain ? 3 : 4) && k <= 8 && bytes >= kWindowMidBytes && bytes < kWindowTunedBytes;
}
// Element-aligned destinations with sources at other phases take reduce_windows_kernel instead of the phased
// kernels where it led by >= 2 points: from kWindowTunedBytes at k-way k = 3..5, chain k = 4..7; mid-size with
// the destination 16-B aligned.
constexpr bool phased_via_windows(bool chain, int k, size_t bytes, bool dst16) {
    if (bytes >= kWindowTunedBytes) return k >= (chain ? 4 : 3) && k <= (chain ? 7 : 5);
    return dst16 && window_mid(chain, k, bytes);
}

// ---- checks of the tables, at every build ----
constexpr bool table_ok() {
    for (int c = 0; c < kNumKernels; ++c)
        for (int s = 0; s < kSizeClasses; ++s)
            for (int k = 0; k <= 8; ++k) {
                const int w = kWaves[c][s][k];
                const bool in_range = k >= min_k(Kernel(c)) && k <= max_k(Kernel(c));
                const bool phased = c == kMultiPhasedFirst || c == kChainPhasedFirst;
                if (!in_range && w != 0) return false;                               // unused cells empty
                if (in_range && !phased && (w < 7 || w > kUncapped)) return false;  // a legal cap
                if (phased && w != 0 && (w < 7 || w > kUncapped)) return false;
                if (phased && (w == 0) != (kWaves[c][3][k] == 0)) return false;     // one form per k
                if (lds_for_waves(w) > kMaxLdsPerBlock) return false;
                const int run = kRun[c][k];
                if (run != 1 && run != 2 && run != 4 && run != 8) return false;  // run_tile's groups
                if (run != 1 && phased && w == 0) return false;                  // a run only for the loads-first form
            }
    for (const auto& row : kWindow)
        for (const WindowForm& f : row)  // legal orders and caps; the loads-first tile only under a cap
            if (f.order > 3 || f.first > 1 || f.waves < 7 || f.waves > kUncapped || (f.first && f.waves == kUncapped))
                return false;
    return true;
}
static_assert(table_ok(), "every cap is a legal LDS request; runs and loads-first tiles only where capped");

}  // namespace caps
}  // namespace dccl_amd
