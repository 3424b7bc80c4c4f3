/*
 * oracle/host_reduce.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of DCCL's host-side local combine
 *     recv[i] = op(recv[i], send[i]),  i in [0, count)
 * as implemented by `do_host_reduce<DT>` in
 *     /root/reference/src/core/internal_common.hpp:496-586
 * with the dtype dispatch of `ON_DCCL_DATATYPE` (internal_common.hpp:350-413).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this file's library, and only as the checker / the timed CPU baseline.
 * The product path (dccl_amd/) never links or calls it.
 *
 * Parity unpinned: the reference holds no test vectors and its
 * combine does not build here without stand-ins (the CMake-generated
 * dccl/config.h and spdlog are absent), so nothing is compiled from
 * /root/reference.  tests/test_oracle.py checks this restatement against
 * regression fixtures in tests/golden/ that were frozen from a round-1 build
 * with stand-in headers (tests/golden/make_golden.py says how; they pin
 * nothing), against the C1 known answers recorded in SURVEY.md §8(c), and
 * against numpy / torch for fp16 / bf16.
 *
 * Two entry points:
 *   oracle_host_reduce()   — the reference's loop split, faithfully: head up to
 *                            the 64-B cache-line boundary of `recv`, packs of
 *                            64/sizeof(T) elements, tail walked backwards from
 *                            the end (internal_common.hpp:531-560).  This
 *                            includes the reference's misalignment overrun
 *                            (SURVEY.md Appendix A.4): with a misaligned `recv`
 *                            and count%P < head it touches P elements past
 *                            `count`.  Callers must pad buffers for such cases.
 *   oracle_expected_reduce() — the combine's intended semantics, one plain pass
 *                            over [0,count).  Identical to oracle_host_reduce
 *                            whenever the A.4 condition does not trigger; this
 *                            is what the HIP path is specified to produce.
 *
 * Per-element semantics (internal_common.hpp:546-549):
 *   Sum  r = r + s        Prod r = r * s      (ints wrap; i8/u8 truncate)
 *   Max  if (r < s) r = s Min  if (r > s) r = s  (NaN or +-0 ties keep r)
 *   Avg  -> ncclInvalidUsage (5), nothing written  (internal_common.hpp:577-580)
 *   op >= 5 -> ncclInvalidArgument (4)             (internal_common.hpp:581-583)
 * Types the reference host path lacks ("parity unpinned" by the
 * reference; cross-checked against numpy float16 / torch bfloat16 instead):
 *   fp16 (6) / bf16 (9): widen both operands to fp32, apply the op, round back
 *   to nearest-even.  Max/Min select the original operand bits.
 * Unknown dtype: the reference silently skips (A.3 #4); this oracle returns 4
 * (ncclInvalidArgument), the documented build contract.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#define ORACLE_CACHELINE 64 /* CACHELINE_SIZE from getconf on x86 (CMakeLists.txt:17-19) */

enum { R_SUCCESS = 0, R_INVALID_ARGUMENT = 4, R_INVALID_USAGE = 5 };
enum { OP_SUM = 0, OP_PROD = 1, OP_MAX = 2, OP_MIN = 3, OP_AVG = 4 };
enum {
    DT_I8 = 0, DT_U8 = 1, DT_I32 = 2, DT_U32 = 3, DT_I64 = 4, DT_U64 = 5,
    DT_F16 = 6, DT_F32 = 7, DT_F64 = 8, DT_BF16 = 9
};

/* ---------------- fp16 / bf16 <-> fp32, round-to-nearest-even ---------------- */

static float f32_from_bits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t bits_from_f32(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

static float half_to_float(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t exp = (h >> 10) & 0x1f;
    uint32_t man = h & 0x3ffu;
    if (exp == 0x1f) /* inf / nan: keep payload */
        return f32_from_bits(sign | 0x7f800000u | (man << 13));
    if (exp == 0) {
        if (man == 0) return f32_from_bits(sign);
        /* subnormal: value = man * 2^-24, exact in fp32 */
        float v = (float)man * 5.9604644775390625e-08f;
        return sign ? -v : v;
    }
    return f32_from_bits(sign | ((exp + 112u) << 23) | (man << 13));
}

static uint16_t float_to_half(float f) {
    uint32_t u = bits_from_f32(f);
    uint16_t sign = (uint16_t)((u >> 16) & 0x8000u);
    uint32_t aexp = (u >> 23) & 0xff;
    uint32_t man = u & 0x7fffffu;
    if (aexp == 0xff) { /* inf / nan (nan stays nan, quiet bit forced) */
        if (man == 0) return sign | 0x7c00u;
        return sign | 0x7e00u | (uint16_t)(man >> 13);
    }
    int32_t e = (int32_t)aexp - 127 + 15;
    if (e >= 0x1f) return sign | 0x7c00u; /* overflow -> inf */
    if (e <= 0) {
        /* result is subnormal or zero: shift full significand into place */
        if (e < -10) return sign; /* below half of the smallest subnormal */
        uint32_t full = man | 0x800000u;
        uint32_t shift = (uint32_t)(14 - e); /* 13 + (1 - e) */
        uint32_t q = full >> shift;
        uint32_t rem = full & ((1u << shift) - 1u);
        uint32_t halfway = 1u << (shift - 1);
        if (rem > halfway || (rem == halfway && (q & 1u))) q++;
        return sign | (uint16_t)q; /* q may carry into the exponent field: correct */
    }
    uint32_t q = ((uint32_t)e << 10) | (man >> 13);
    uint32_t rem = man & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (q & 1u))) q++; /* may round up to inf: correct */
    return sign | (uint16_t)q;
}

static float bf16_to_float(uint16_t b) { return f32_from_bits((uint32_t)b << 16); }

static uint16_t float_to_bf16(float f) {
    uint32_t u = bits_from_f32(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) /* nan: keep sign/payload top bits, force quiet */
        return (uint16_t)((u >> 16) | 0x0040u);
    uint32_t lsb = (u >> 16) & 1u;
    return (uint16_t)((u + 0x7fffu + lsb) >> 16);
}

/* ---------------- per-element operators ---------------- */

/* Integer arithmetic goes through the unsigned type of the same width so that
 * wrap-around is defined behaviour in C; the bit results equal the reference's
 * (gcc, two's complement).  8-bit types promote to int and truncate on store,
 * exactly as `r += s` / `r *= s` on int8_t/uint8_t do. */
#define DEF_INT_OPS(NAME, T, UT)                                                   \
    static inline void NAME##_sum(T* r, const T* s) { *r = (T)(UT)((UT)*r + (UT)*s); } \
    static inline void NAME##_prod(T* r, const T* s) { *r = (T)(UT)((UT)*r * (UT)*s); } \
    static inline void NAME##_max(T* r, const T* s) { if (*r < *s) *r = *s; }      \
    static inline void NAME##_min(T* r, const T* s) { if (*r > *s) *r = *s; }

DEF_INT_OPS(i8, int8_t, uint32_t)
DEF_INT_OPS(u8, uint8_t, uint32_t)
DEF_INT_OPS(i32, int32_t, uint32_t)
DEF_INT_OPS(u32, uint32_t, uint32_t)
DEF_INT_OPS(i64, int64_t, uint64_t)
DEF_INT_OPS(u64, uint64_t, uint64_t)

#define DEF_FP_OPS(NAME, T)                                                        \
    static inline void NAME##_sum(T* r, const T* s) { *r = *r + *s; }              \
    static inline void NAME##_prod(T* r, const T* s) { *r = *r * *s; }             \
    static inline void NAME##_max(T* r, const T* s) { if (*r < *s) *r = *s; }      \
    static inline void NAME##_min(T* r, const T* s) { if (*r > *s) *r = *s; }

DEF_FP_OPS(f32, float)
DEF_FP_OPS(f64, double)

#define DEF_HALF_OPS(NAME, TO_F, FROM_F)                                           \
    static inline void NAME##_sum(uint16_t* r, const uint16_t* s)                  \
        { *r = FROM_F(TO_F(*r) + TO_F(*s)); }                                      \
    static inline void NAME##_prod(uint16_t* r, const uint16_t* s)                 \
        { *r = FROM_F(TO_F(*r) * TO_F(*s)); }                                      \
    static inline void NAME##_max(uint16_t* r, const uint16_t* s)                  \
        { if (TO_F(*r) < TO_F(*s)) *r = *s; }                                      \
    static inline void NAME##_min(uint16_t* r, const uint16_t* s)                  \
        { if (TO_F(*r) > TO_F(*s)) *r = *s; }

DEF_HALF_OPS(f16, half_to_float, float_to_half)
DEF_HALF_OPS(bf16, bf16_to_float, float_to_bf16)

/* ---------------- loop shapes ---------------- */

/* Faithful loop split of internal_common.hpp:531-560. */
#define SPLIT_LOOP(T, FN)                                                          \
    do {                                                                           \
        const T* ps = (const T*)send;                                              \
        T* pr = (T*)recv;                                                          \
        size_t head = (ORACLE_CACHELINE - (uintptr_t)recv % ORACLE_CACHELINE)      \
                      % ORACLE_CACHELINE / sizeof(T);                              \
        const size_t pack = ORACLE_CACHELINE / sizeof(T);                          \
        size_t npack = count / pack;                                               \
        size_t tail = (pack + count % pack - head) % pack;                         \
        if (tail + head > count) { head = count; tail = 0; }                       \
        for (size_t i = 0; i < head; i++) FN(&pr[i], &ps[i]);                      \
        for (size_t j = 0; j < npack; j++)                                         \
            for (size_t i = 0; i < pack; i++)                                      \
                FN(&pr[head + j * pack + i], &ps[head + j * pack + i]);            \
        for (size_t i = 0; i < tail; i++)                                          \
            FN(&pr[count - 1 - i], &ps[count - 1 - i]);                            \
    } while (0)

#define PLAIN_LOOP(T, FN)                                                          \
    do {                                                                           \
        const T* ps = (const T*)send;                                              \
        T* pr = (T*)recv;                                                          \
        for (size_t i = 0; i < count; i++) FN(&pr[i], &ps[i]);                     \
    } while (0)

#define DISPATCH_OP(LOOP, T, NAME)                                                 \
    switch (op) {                                                                  \
    case OP_SUM: LOOP(T, NAME##_sum); break;                                       \
    case OP_PROD: LOOP(T, NAME##_prod); break;                                     \
    case OP_MAX: LOOP(T, NAME##_max); break;                                       \
    case OP_MIN: LOOP(T, NAME##_min); break;                                       \
    case OP_AVG: return R_INVALID_USAGE;                                           \
    default: return R_INVALID_ARGUMENT;                                            \
    }

#define DISPATCH_ALL(LOOP)                                                         \
    switch (dtype) {                                                               \
    case DT_I8: DISPATCH_OP(LOOP, int8_t, i8) break;                               \
    case DT_U8: DISPATCH_OP(LOOP, uint8_t, u8) break;                              \
    case DT_I32: DISPATCH_OP(LOOP, int32_t, i32) break;                            \
    case DT_U32: DISPATCH_OP(LOOP, uint32_t, u32) break;                           \
    case DT_I64: DISPATCH_OP(LOOP, int64_t, i64) break;                            \
    case DT_U64: DISPATCH_OP(LOOP, uint64_t, u64) break;                           \
    case DT_F16: DISPATCH_OP(LOOP, uint16_t, f16) break;                           \
    case DT_F32: DISPATCH_OP(LOOP, float, f32) break;                              \
    case DT_F64: DISPATCH_OP(LOOP, double, f64) break;                             \
    case DT_BF16: DISPATCH_OP(LOOP, uint16_t, bf16) break;                         \
    default: return R_INVALID_ARGUMENT;                                            \
    }                                                                              \
    return R_SUCCESS;

int oracle_host_reduce(const void* send, void* recv, size_t count, int dtype, int op) {
    DISPATCH_ALL(SPLIT_LOOP)
}

int oracle_expected_reduce(const void* send, void* recv, size_t count, int dtype, int op) {
    DISPATCH_ALL(PLAIN_LOOP)
}

/* Conversions exported for the tests' own cross-checks against numpy / torch. */
float oracle_half_to_float(uint16_t h) { return half_to_float(h); }
uint16_t oracle_float_to_half(float f) { return float_to_half(f); }
float oracle_bf16_to_float(uint16_t b) { return bf16_to_float(b); }
uint16_t oracle_float_to_bf16(float f) { return float_to_bf16(f); }

/* ---------------- synthetic operands ----------------
 * Host restatement of the generator documented in include/dccl/dccl_synth.h; the tests use it
 * to regenerate full-size operands and check the device combine bit for bit.  Written from the
 * published splitmix64 finaliser (Steele, Lea, Flood 2014), independently of the HIP kernel. */
static uint64_t splitmix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

int oracle_synth_fill(void* dst, int dtype, size_t count, int op, uint64_t seed, uint64_t buffer_id,
                      size_t first) {
    const uint64_t key = seed ^ (buffer_id << 40);
    const int prod = op == OP_PROD;
    for (size_t j = 0; j < count; j++) {
        const uint64_t x = splitmix64(key ^ (uint64_t)(first + j));
        switch (dtype) {
        case DT_I8: case DT_U8: ((uint8_t*)dst)[j] = (uint8_t)x; break;
        case DT_I32: case DT_U32: ((uint32_t*)dst)[j] = (uint32_t)x; break;
        case DT_I64: case DT_U64: ((uint64_t*)dst)[j] = x; break;
        case DT_F32:
            if (prod) ((uint32_t*)dst)[j] = (uint32_t)(((126u + (x >> 63)) << 23) | (x & 0x7fffffu));
            else ((float*)dst)[j] = (float)((int32_t)(x >> 40) - (1 << 23)) / 8388608.0f;
            break;
        case DT_F64:
            if (prod) ((uint64_t*)dst)[j] = ((1022ull + (x >> 63)) << 52) | (x & 0xfffffffffffffull);
            else ((double*)dst)[j] = (double)((int64_t)(x >> 11) - (1ll << 52)) / 4503599627370496.0;
            break;
        case DT_F16:
            if (prod) ((uint16_t*)dst)[j] = (uint16_t)(((14u + (x >> 63)) << 10) | (x & 0x3ffu));
            else ((uint16_t*)dst)[j] = float_to_half((float)((int32_t)(x >> 53) - (1 << 10)) / 1024.0f);
            break;
        case DT_BF16:
            if (prod) ((uint16_t*)dst)[j] = (uint16_t)(((126u + (x >> 63)) << 7) | (x & 0x7fu));
            else ((uint16_t*)dst)[j] = float_to_bf16((float)((int32_t)(x >> 56) - (1 << 7)) / 128.0f);
            break;
        default: return R_INVALID_ARGUMENT;
        }
    }
    return R_SUCCESS;
}
