// dccl_amd/csrc/caps.hpp — resident-wave caps of every capped combine launch, in one table, and the one
// function that selects them.  Pure host C++ (no HIP): tests/test_caps.py compiles it with g++ and checks
// every entry; the static_asserts below check the table at every build.
//
// Why caps.  Every combine kernel is a one-wave (64-thread) block streaming 16-B vectors.  A CU holds up
// to 32 such blocks; with k + 1 loads per lane in flight each, too many bytes are outstanding and the DRAM
// serves the streams worse.  A launch asks for `bytes` of (unused) dynamic LDS per block, so a CU holds
// floor(160 KiB / bytes) of them (lds_for_waves).  The values are NOMINAL wave counts: the 256-B rounding
// of the LDS request makes some neighbours the same occupancy (8 and 9, 16 and 18).
//
// How they were chosen (profiles/): each entry is the best cap of a sweep of the launch at
// that k, 1 GiB fp32 Sum per operand for the 1 GiB row, operand sets rotated past the Infinity Cache for
// the size rows; a size-row entry differs from the 1 GiB row only where that gained at least one point.
// Frozen from round 3: an entry changes only for a candidate that leads by >= 2 points on two boxes.
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

inline constexpr int kUncapped = 32;          // 32 one-wave blocks per CU: the hardware limit
inline constexpr size_t kLdsPerCu = size_t(160) << 10;
inline constexpr size_t kMaxLdsPerBlock = size_t(64) << 10;
inline constexpr int kSizeClasses = 4;

// Size class of a launch by bytes per operand: 0, 1, 2 below 24, 48 and 96 MiB, 3 (the 1 GiB-tuned row)
// from 96 MiB.  Below 96 MiB a launch has few tiles per resident wave and its tail dominates, so more
// resident waves win.
constexpr int size_class(size_t bytes) {
    return bytes < (size_t(24) << 20) ? 0 : bytes < (size_t(48) << 20) ? 1 : bytes < (size_t(96) << 20) ? 2 : 3;
}

// kWaves[kernel][size class][k]: nominal resident waves per CU (32 = uncapped; 0 = the kernel class is
// not used at that k).  Evidence per row:
//  kMulti      1 GiB: r1 sweep (+3-5 points over uncapped, r1_tune_multi_waves.json), r2 re-sweep at 1 GiB on
//              both layouts found nothing 0.7 points better (r2_kway_waves.json); size rows: kway_size_caps.py,
//              +1 to +8 points at 16-64 MiB (r2_s70_kway_size_caps_*.json, two sweeps within 0.2 points).
//  kChain      as kMulti (r1_s5_chain_waves_sweep.json, r2_kway_waves.json, r2_s70_kway_size_caps_*.json).
//  kMultiStraddle / kChainStraddle  phased_probe.py --straddle-caps (r2_kway_straddle_caps.json; A/B on a
//              second box r2_kway_straddle_caps_ab.json: k-way k = 6 74.1 -> 79.0 %, chain k = 4 77.3 ->
//              80.2 %); size rows r2_s70_kway_size_caps_straddle*.json.
//  kMultiPhasedFirst / kChainPhasedFirst  the loads-first form wins from k = 5 (k-way) / k = 4 (chain)
//              under these caps on two boxes (r2_phased_first_caps.json, r2_phased_first_ab.json); size rows
//              r2_s70_..._phased.json.  Round 3: in the tile-run order of kRun the loads-first form also wins at
//              k-way k = 4, 6 and chain k = 3, and the k-way k = 7, 8 / chain k = 7 caps move to 13 (+2.0 to
//              +3.7 points on two boxes, r3_s11_runs_straddle_phased.json, r3_s12_runs_confirm_*.json,
//              r3_s10_phased_run_orders.json); their size rows take the 1 GiB value (not swept).
//  kMultiStraddle k = 8: 9 waves in kRun's order (+2.4 to +3.3 on four boxes, r3_s9..s12).
// The misaligned-recv kernel took a cap of its own in round 2 (24 waves); round 3's form (recv read through
// aligned loads, group-interleaved tile order) runs best uncapped (profiles/r3_s4_unaligned_orders_caps.json),
// so that row is gone.
inline constexpr unsigned char kWaves[kNumKernels][kSizeClasses][9] = {
    // k:  0   1   2   3   4   5   6   7   8
    {{0, 0, 32, 24, 16, 16, 16, 16, 32},  // kMulti            < 24 MiB
     {0, 0, 32, 20, 16, 16, 11, 10, 9},   //                   < 48 MiB
     {0, 0, 24, 16, 13, 11, 11, 10, 9},   //                   < 96 MiB
     {0, 0, 18, 13, 13, 11, 11, 10, 9}},  //                   from 96 MiB
    {{0, 32, 32, 32, 32, 24, 16, 16, 16},  // kChain
     {0, 32, 32, 32, 16, 16, 16, 16, 16},
     {0, 32, 32, 24, 16, 13, 11, 10, 9},
     {0, 32, 24, 20, 16, 13, 11, 10, 9}},
    {{0, 0, 32, 24, 16, 16, 16, 16, 32},  // kMultiStraddle
     {0, 0, 24, 16, 13, 11, 16, 9, 32},
     {0, 0, 24, 16, 13, 11, 9, 9, 9},
     {0, 0, 18, 13, 13, 11, 9, 9, 9}},
    {{0, 32, 32, 32, 24, 24, 16, 16, 16},  // kChainStraddle
     {0, 32, 32, 32, 24, 16, 11, 10, 9},
     {0, 32, 32, 24, 16, 13, 11, 10, 9},
     {0, 32, 24, 18, 13, 13, 11, 10, 9}},
    {{0, 0, 0, 0, 16, 16, 13, 24, 16},  // kMultiPhasedFirst
     {0, 0, 0, 0, 16, 16, 13, 16, 24},
     {0, 0, 0, 0, 16, 13, 13, 13, 13},
     {0, 0, 0, 0, 16, 13, 13, 13, 13}},
    {{0, 0, 0, 16, 24, 24, 0, 24, 16},  // kChainPhasedFirst
     {0, 0, 0, 16, 16, 16, 0, 16, 24},
     {0, 0, 0, 16, 16, 13, 0, 13, 11},
     {0, 0, 0, 16, 13, 13, 0, 13, 11}},
};

// kRun[kernel][k]: the tile-run order of the launch (reduce_kernels.hpp run_tile<RUN>: each XCD walks RUN
// consecutive tiles of every group of 8 RUN blocks; 1 = block order).  Runs of 4 keep the chip on one front
// while the line two neighbouring tiles share (lane 63's extra load of an off-phase operand, a straddling
// source's partial line) is fetched by one L2 in 3 of 4 cases (round 3, the files above).  The phased
// per-operand form (kPhasedXcdMaxK) keeps consecutive tiles on one XCD and is not covered by this table.
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

// Nominal waves of a launch of class c with k sources and `bytes` per operand; -1 for a k outside the
// class's range.  0 for the phased classes means "the per-operand form, uncapped".
constexpr int waves(Kernel c, int k, size_t bytes) {
    return (c < 0 || c >= kNumKernels || k < min_k(c) || k > max_k(c)) ? -1 : kWaves[c][size_class(bytes)][k];
}

// Dynamic LDS bytes per one-wave block for a nominal wave count (0 = no request: uncapped).
constexpr size_t lds_for_waves(int w) { return (w <= 0 || w >= kUncapped) ? 0 : (kLdsPerCu / size_t(w) + 255) / 256 * 256; }

// The LDS request of a launch (0 = uncapped, also for a k outside the class's range).
constexpr size_t lds(Kernel c, int k, size_t bytes) { return lds_for_waves(waves(c, k, bytes)); }

// Does the phased k-way (chain) launch with k sources take the loads-first form?  A compile-time choice
// per K: the 1 GiB row decides (every size row agrees on which k are non-zero, checked below).
constexpr bool phased_loads_first(bool chain, int k) {
    return waves(chain ? kChainPhasedFirst : kMultiPhasedFirst, k, size_t(1) << 30) > 0;
}

// Pairwise launches: capped only when send and recv lie in two allocations of at least kSeparateCapBytes
// each on the current device (DCCL's scratchpad + user chunk).  Paired A/B of the same pairs under every
// cap (separate_cap_paired.py@4f20423, 6-8 separate pairs per run, profiles/r2_s61_separate_cap_*.json,
// r2_s66_separate_cap_shift*.json), median pair against uncapped: aligned at 22 resident waves +0.6 to
// +1.0 points at 1 GiB (six runs, three boxes), -0.8 at 256 MiB; shifted at 26 +1.0 to +1.25 (four runs);
// one-allocation pairs lose 0.4-1.1 under any cap and stay uncapped.  The LDS bytes are the values measured.
inline constexpr size_t kSeparateCapBytes = size_t(512) << 20;
inline constexpr size_t kSeparateLds = 7168;       // aligned vector kernel: floor(160 KiB / 7168) = 22 waves
inline constexpr size_t kSeparateShiftLds = 6144;  // shifted kernel: 26 waves

constexpr size_t pair_lds(bool shifted, bool separate_allocations, size_t bytes) {
    return (!separate_allocations || bytes < kSeparateCapBytes) ? 0 : shifted ? kSeparateShiftLds : kSeparateLds;
}

// ---- reduce_windows_kernel (k-way / chain into a destination read and written at its own 16-B phase) ----
// Round 4: the per-operand form runs K + 1 dependent load round trips per tile and wants a
// cap like the other k-way kernels; with sources off phase the loads-first form under a lower cap wins at
// k = 4, 5.  tools/ab_unaligned.py, 1 GiB fp32 Sum, destination + 2 B, 5 rounds, against the uncapped form
// (profiles/r4_s11_ab_first.json, r4_s12_*.json, r4_s13_ab_forms.json, three boxes):
//   sources in phase, per-operand, block order, 26 waves: k = 3 +3.5, 4 +2.6..+3.2, 5 +2.1, 6 +1.1,
//     7 +0.9, 8 +0.7..+1.2 points (k <= 2 keeps the round-3 kernels, unaligned_multi.hip);
//   sources off phase: k = 3 per-operand, group-interleaved order, 26 waves +1.9..+3.7; k = 4 loads-first,
//     group order, 14 waves +4.9..+5.3; k = 5 the same at 12 +4.6; k = 6..8 loads-first in runs of 4 tiles
//     (run_tile<4>) at 13 waves: k = 6, 7 +2.5..+3.6, k = 8 +0.5..+1.2 (r4_s17_ab_runs.json, r4_s18_ab_runs2.json).
// PMC traffic stays within 2 % of (k+1)·N reads and N writes (k = 8 sources + 4 B: 1.02 x, r4_s18_pmc/): what
// is left at k = 8 off phase (75 %) is how the DRAM serves ten concurrent streams, not re-reads.
// The same forms beat the phased kernels (element-aligned destination, sources at other phases) at k-way
// k = 3..5 (+1.2..+2.8, +4.2..+5.0, +2.9..+4.3) and chain k = 4..7 (+4.2..+5.0, +2.8..+4.3, +2.9..+3.0,
// +1.9..+2.1): those launches take reduce_windows_kernel too (phased_via_windows).  Not the chain at k = 3
// (-0.8..-1.1 with the destination off the line grid, r4_s15_ab_windows_forms.json), nor k-way k = 6, 7
// (+0.4..+1.0, below the 2-point bar), nor k = 8 (the phased kernels lead).
// From kWindowMidBytes to kWindowTunedBytes per operand (r4_s20_ab_64mib.json; 64-88 MiB A/B of the shipped
// build, r4_s26_ab_mid*.json, r4_s27_ab_mid*_k34.json), sources off phase: k = 4..8 the loads-first tile in
// group order under 14 waves, +0.0..+2.6 points into a misaligned destination and +3.0..+6.6 over the phased
// kernels (element-aligned destination at 16-B phase 0); the chain at k = 3 per-operand in group order under
// 26 waves (+4.9..+6.0 over the phased kernel; the k-way at k = 3 lost 0.3-3.8 and keeps its kernels);
// everything else there, and every launch below kWindowMidBytes, keeps the uncapped per-operand form.
inline constexpr size_t kWindowTunedBytes = size_t(96) << 20;
inline constexpr size_t kWindowMidBytes = size_t(48) << 20;
inline constexpr int kWindowMidMinK = 4;  // k-way; the chain from k = 3
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
inline constexpr WindowForm kWindowMidOff[9] = {{0, 0, 32}, {0, 0, 32}, {0, 0, 32}, {0, 2, 26}, {1, 2, 14},
                                                 {1, 2, 14}, {1, 2, 14}, {1, 2, 14}, {1, 2, 14}};
constexpr WindowForm window_mid_form(int k) { return kWindowMidOff[k < 0 ? 0 : k > 8 ? 8 : k]; }
constexpr bool window_mid(bool chain, int k, size_t bytes) {
    return k >= (chain ? 3 : kWindowMidMinK) && k <= 8 && bytes >= kWindowMidBytes && bytes < kWindowTunedBytes;
}
// Element-aligned destinations with sources at other phases: reduce_windows_kernel's tuned form instead of
// the phased kernels, from kWindowTunedBytes; and its mid-size form (window_mid) for a destination at 16-B
// phase 0 (so some source is off phase).
constexpr bool phased_via_windows(bool chain, int k, size_t bytes, bool dst16 = false) {
    if (bytes >= kWindowTunedBytes) return k >= (chain ? 4 : 3) && k <= (chain ? 7 : 5);
    return dst16 && window_mid(chain, k, bytes);
}
// Straddling sources (every operand at the 16-B aligned destination's phase, some off its 128-B lines): the
// mid-size window form (window_mid_form) instead of the straddle kernels in a per-k size band.  The window
// form runs flat at 77-80 % of (k+2)·N from 48 to 96 MiB; the straddle kernels climb with size at k = 7, 8,
// so the band ends where they catch up.  tools/ab_cases.py, shipped build against the build with this route
// from 48 to 96 MiB at k = 5..8, fp32 Sum, 7 rounds, two boxes (profiles/r4_s31_ab_strad*.json at 48/64/88
// MiB, r4_s32_ab_strad*.json at 56/64/72/80/88 MiB), k-way / chain: k = 5 from 72 MiB +2.2..+3.3 / +2.5..+3.0
// (64 MiB +0.1..+0.7); k = 6 from 56 MiB +2.8..+5.0 / +1.2..+2.0 (48 MiB -0.4..+0.2); k = 7 56-80 MiB
// +1.3..+3.0 / +0.6..+3.1 (88 MiB +0.6..+1.7); k = 8 56-72 MiB +2.1..+4.2 / +0.8..+3.9 (80 MiB -0.8..+1.2,
// 88 MiB -1.5..-0.5).  Every result bit-exact against the straddle kernels.
struct MibBand { unsigned short lo, hi; };  // [lo, hi) MiB per operand
inline constexpr MibBand kStradMid[9] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {72, 96}, {56, 96}, {56, 80}, {56, 72}};
constexpr bool strad_via_windows(int k, size_t bytes) {
    if (k < 0 || k > 8) return false;
    const MibBand b = kStradMid[k];
    return bytes >= (size_t(b.lo) << 20) && bytes < (size_t(b.hi) << 20);
}

// ---- checks of the table, at every build ----
constexpr bool table_ok() {
    for (int c = 0; c < kNumKernels; ++c)
        for (int s = 0; s < kSizeClasses; ++s)
            for (int k = 0; k <= 8; ++k) {
                const int w = kWaves[c][s][k];
                const bool in_range = k >= min_k(Kernel(c)) && k <= max_k(Kernel(c));
                const bool phased = c == kMultiPhasedFirst || c == kChainPhasedFirst;
                if (!in_range && w != 0) return false;                                  // unused cells empty
                if (in_range && !phased && (w < 7 || w > kUncapped)) return false;     // a legal cap
                if (phased && w != 0 && (w < 7 || w > kUncapped)) return false;
                if (phased && (w == 0) != (kWaves[c][3][k] == 0)) return false;         // one form per k
                if (lds_for_waves(w) > kMaxLdsPerBlock) return false;
                const int run = kRun[c][k];
                if (run != 1 && run != 2 && run != 4 && run != 8) return false;  // run_tile's groups
                if (run != 1 && phased && w == 0) return false;  // a run only for the loads-first form
            }
    return true;
}
static_assert(table_ok(), "every cap is a legal LDS request and the phased form is fixed per k");
constexpr bool window_table_ok() {
    for (int c = 0; c < kNumWindowClasses; ++c)
        for (int k = 0; k <= 8; ++k) {
            const WindowForm f = kWindow[c][k];
            if (f.order > 3 || f.first > 1 || f.waves < 7 || f.waves > kUncapped) return false;
            if (f.first && f.waves == kUncapped) return false;  // the loads-first tile only under a cap
            if (lds_for_waves(f.waves) > kMaxLdsPerBlock) return false;
        }
    for (int k = 3; k <= 7; ++k)  // the phased launches routed to the windows kernel take a tuned off-phase form
        if (kWindow[kWinOffPhase][k].waves == kUncapped) return false;
    return true;
}
static_assert(window_table_ok(), "window forms: legal orders and caps, loads-first only capped");
constexpr bool strad_table_ok() {
    for (int k = 0; k <= 8; ++k) {
        const MibBand b = kStradMid[k];
        if (b.lo == b.hi) continue;
        // inside window_mid's range, where launch_windows takes the mid-size form
        if (b.lo >= b.hi || (size_t(b.lo) << 20) < kWindowMidBytes || (size_t(b.hi) << 20) > kWindowTunedBytes ||
            k < kWindowMidMinK)
            return false;
    }
    return true;
}
static_assert(strad_table_ok(), "straddle bands lie inside the mid-size window range");
static_assert(size_class((size_t(24) << 20) - 1) == 0 && size_class(size_t(24) << 20) == 1 &&
                  size_class(size_t(48) << 20) == 2 && size_class(size_t(96) << 20) == 3,
              "size-class boundaries at 24 / 48 / 96 MiB");
static_assert(kLdsPerCu / kSeparateLds == 22 && kLdsPerCu / kSeparateShiftLds == 26, "pair caps");

}  // namespace caps
}  // namespace dccl_amd
