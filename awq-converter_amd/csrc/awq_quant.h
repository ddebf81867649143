// awq_quant.h — device helpers shared by the streaming kernel (awq_fast.hip) and the
// row-segment kernel (awq_rowgroup.hip): input formats (raw-bits min/max, decoding, the
// reference's per-op rounding and exact quotients), group parameters from a group's range
// (awq.py:173-213), the field chain and nibble / byte packing (awq.py:215-250), fp16 scale
// bits (awq.py:411).  Each including file gets its own copies (anonymous namespace).
#ifndef AWQ_QUANT_H
#define AWQ_QUANT_H
#include <cstdlib>
#include <type_traits>

#include "awq_internal.h"

// Cache-policy bits of the input loads and the qweight / tensor_q stores (gfx950: 2 = nt).
#define AWQ_LOAD_AUX 2
#define AWQ_STORE_AUX 2
// Cache policy of the small per-tile stores (scales, zeros, qzeros: 8-32 B per tile).
// Default policy (0), not nt: the L2 then merges the partial lines neighbouring tiles
// write (measured +2-5 % over nt, profiles/r19-r20)
#define AWQ_SMALL_AUX 0
// __launch_bounds__ minimum waves per SIMD (8 = 32 waves per CU: <= 64 VGPRs, <= 80 SGPRs)
#define AWQ_MIN_WAVES 8
// same for fp32 inputs (32 data VGPRs per lane instead of 16)
#define AWQ_MIN_WAVES_WIDE 6

namespace awq {
namespace {

typedef short s2 __attribute__((ext_vector_type(2)));
typedef unsigned short us2 __attribute__((ext_vector_type(2)));
typedef float f2 __attribute__((ext_vector_type(2)));
// two-element f32 ops (v_pk_mul_f32 / v_pk_add_f32 where the compiler keeps the pair packed)
__device__ __forceinline__ f2 pk_mul(f2 a, f2 b) { return a * b; }
__device__ __forceinline__ f2 pk_add(f2 a, f2 b) { return a + b; }
typedef __bf16 b2 __attribute__((ext_vector_type(2)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
typedef uint32_t u2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes,
                                             0x00020000);
}

__device__ __forceinline__ s2 as_s2(uint32_t u) { return __builtin_bit_cast(s2, u); }
__device__ __forceinline__ us2 as_us2(uint32_t u) { return __builtin_bit_cast(us2, u); }

// RN_bf16 of an fp32 value, returned as fp32: v_cvt_pk_bf16_f32 dst, 0, a puts
// bf16(a) in the high half and zero in the low half — which is bf16(a) as an fp32.
// Hardware RNE; NaN stays NaN.
__device__ __forceinline__ float rn_bf16(float a) {
    b2 h = __builtin_convertvector((f2){0.0f, a}, b2);
    return __builtin_bit_cast(float, h);
}

// one step of a 16-lane row reduction: max with a DPP-permuted copy (full row/bank masks,
// every source lane valid) — LLVM folds the mov into v_max_i32_dpp (one instruction)
template <int CTRL, typename T>
__device__ __forceinline__ T dpp_max(T v) {   // T = int (signed max) or uint32_t (unsigned)
    return max(v, (T)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true));
}

// max over the L = GS/8 consecutive lanes of a group; every lane of the group gets it.
// L <= 16: DPP steps inside a row (each folds into one v_max_i32_dpp); L = 32: the group
// spans two rows, paired by one v_permlane16_swap (gfx950).
template <int L, typename T>
__device__ __forceinline__ T grp_max(T v) {
    static_assert(L == 4 || L == 8 || L == 16 || L == 32, "lanes per group");
    v = dpp_max<0xB1>(v);                  // quad_perm [1,0,3,2]
    v = dpp_max<0x4E>(v);                  // quad_perm [2,3,0,1]
    if (L >= 8) v = dpp_max<0x141>(v);     // row_half_mirror
    if (L >= 16) v = dpp_max<0x140>(v);    // row_mirror
    if (L >= 32) {                         // rows 0<->1, 2<->3
        const auto p = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
        v = max((T)p[0], (T)p[1]);
    }
    return v;
}

// value of lane J of each quad broadcast to its quad (DPP quad_perm [J,J,J,J]).  Every lane
// c of a group with c & 3 == J holds the parameters of the group in load J, so this one
// DPP hands them to all the group's lanes for any GS.
template <int J>
__device__ __forceinline__ float quad_bcast(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), J * 0x55, 0xF, 0xF, true));
}

__device__ __forceinline__ float bcast_j(int j, float v) {   // j is a compile-time constant at every use
    return j == 0 ? quad_bcast<0>(v) : j == 1 ? quad_bcast<1>(v) : j == 2 ? quad_bcast<2>(v) : quad_bcast<3>(v);
}
__device__ __forceinline__ uint32_t bcast_u(int j, uint32_t v) {
    return __builtin_bit_cast(uint32_t, bcast_j(j, __builtin_bit_cast(float, v)));
}

// RN_f32(1/s) for a bf16-valued s: v_rcp_f32 + one Newton step with fma is correctly
// rounded for every bf16 s < 2^126 (checked exhaustively on the GPU by awq_selftest);
// larger, inf and NaN go through the IEEE division.
__device__ __forceinline__ float recip_bf16(float s) {
    if (__builtin_expect(!(s < 0x1p126f), 0)) return 1.0f / s;
    const float r0 = __builtin_amdgcn_rcpf(s);
    const float e = __builtin_fmaf(-s, r0, 1.0f);
    return __builtin_fmaf(r0, e, r0);
}
// The same for an fp16-valued s: correctly rounded for every positive finite fp16 s (all 31 743,
// awq_selftest 2 on the GPU); 0, inf and NaN go through the IEEE division.
__device__ __forceinline__ float recip_f16(float s) {
    if (__builtin_expect(!(s > 0.0f && s < __builtin_inff()), 0)) return 1.0f / s;
    const float r0 = __builtin_amdgcn_rcpf(s);
    const float e = __builtin_fmaf(-s, r0, 1.0f);
    return __builtin_fmaf(r0, e, r0);
}

// ---- input formats ----------------------------------------------------------------
// All are sign-magnitude floats, so the raw-bits min/max below works for each.  They
// differ in width (a lane's 8 consecutive elements of a group are one 16-B load for the
// 16-bit formats, two for fp32), decoding, NaN thresholds, the rounding applied after
// every op (torch computes a bf16/fp16 op in fp32 and rounds to the dtype, awq.py's per-op
// semantics) and in how x / s is formed exactly.
template <int NW>
struct Chunk {
    u4 w[NW];
};

// raw-bits lane maxima of 8 packed 16-bit values: signed (sign-extended) and unsigned
__device__ __forceinline__ void lane_max16(const u4 v, int& smax, uint32_t& umax) {
    // (the bit casts go through by-value helpers: hipcc 7.2 miscompiles
    //  __builtin_bit_cast applied directly to an ext_vector element)
    const uint32_t x0 = v.x, x1 = v.y, x2 = v.z, x3 = v.w;
    const s2 sm = __builtin_elementwise_max(__builtin_elementwise_max(as_s2(x0), as_s2(x1)),
                                            __builtin_elementwise_max(as_s2(x2), as_s2(x3)));
    const us2 um = __builtin_elementwise_max(__builtin_elementwise_max(as_us2(x0), as_us2(x1)),
                                             __builtin_elementwise_max(as_us2(x2), as_us2(x3)));
    smax = max((int)sm.x, (int)sm.y);
    umax = (uint32_t)max((int)um.x, (int)um.y);
}
// max of the complements 0xFFFF - u (unsigned min = 0xFFFF - that)
__device__ __forceinline__ uint32_t lane_cmax16(const u4 v) {
    const us2 ones = {0xFFFF, 0xFFFF};
    const uint32_t x0 = v.x, x1 = v.y, x2 = v.z, x3 = v.w;
    const us2 a = ones - as_us2(x0), b = ones - as_us2(x1);
    const us2 c = ones - as_us2(x2), e = ones - as_us2(x3);
    const us2 m = __builtin_elementwise_max(__builtin_elementwise_max(a, b), __builtin_elementwise_max(c, e));
    return (uint32_t)max((int)m.x, (int)m.y);
}

struct FmtBF16 {
    static constexpr int NW = 1, kBytes = 2;
    static constexpr bool kWide = false;
    static constexpr int kNanS = 0x7F80;                   // bits beyond +inf / -inf
    static constexpr uint32_t kNanU = 0xFF80u, kSign = 0x8000u, kOnes = 0xFFFFu;
    __device__ static void lane_max(const Chunk<1>& c, int& smax, uint32_t& umax) { lane_max16(c.w[0], smax, umax); }
    __device__ static uint32_t lane_cmax(const Chunk<1>& c) { return lane_cmax16(c.w[0]); }
    __device__ static float dec(uint32_t h) { return __uint_as_float(h << 16); }
    __device__ static float lo(uint32_t w) { return __uint_as_float(w << 16); }
    __device__ static float hi(uint32_t w) { return __uint_as_float(w & 0xFFFF0000u); }
    __device__ static float rn(float a) { return rn_bf16(a); }
    __device__ static float as_fmt(float z) { return z; }
    // fp16 value of the scale the reference's dequantize multiplies by (awq.py:411, 459-539)
    __device__ static float dq_scale(float s) { return (float)(_Float16)s; }
    // RN(x / s) for a finite s: RN_bf16(x * RN_f32(1/s)) is exact (oracle/verify_recip.c)
    __device__ static float quot(float x, float s, float r) {
        (void)s;
        return rn_bf16(x * r);
    }
    // awq.py:202 before the clamp: RN(RN(mx - mn) / QR); / QR == * RN(1/QR), same identity
    __device__ static float scale(float d, float qr) { return rn_bf16(rn_bf16(d) * (1.0f / qr)); }
    __device__ static float lo_clamp() { return __uint_as_float(0x2EDC0000u); }   // RN_bf16(1e-10)
    __device__ static float recip(float s) { return recip_bf16(s); }
    // awq.py:210 RN(mn / s) for the zero point, any s (r = 0 for s = inf, NaN for NaN)
    __device__ static float quot_any(float x, float s, float r) { return quot(x, s, r); }
    // the per-element fast path needs a finite scale (s >= 1e-10 always)
    __device__ static bool fast(float r) { return r > 0.0f; }
    // quot() is already the plain product
    static constexpr bool kHasPlain = false;
    __device__ static bool plain_ok(float s) { (void)s; return false; }
    __device__ static float quot_plain(float x, float r) { return rn_bf16(x * r); }
    __device__ static float elem(const Chunk<1>& c, int i) {
        const uint32_t w = c.w[0][i >> 1];
        return (i & 1) ? hi(w) : lo(w);
    }
};

// An f32 value the optimizer cannot see through: keeps `RN_f16(a / b)` an f32 IEEE division
// followed by one v_cvt_f16_f32, instead of being narrowed to an f16 division (whose
// rcp-based lowering we do not rely on for exactness).
__device__ __forceinline__ float opaque(float a) {
    asm volatile("" : "+v"(a));
    return a;
}

// same for a wave-uniform constant kept in an SGPR (usable as a VOP3P operand in place)
__device__ __forceinline__ float opaque_s(float a) {
    asm("" : "+s"(a));   // not volatile: one copy per kernel, hoisted
    return a;
}

// AWQ_F16_PARAMS_FAST = 0: the fp16 group parameters by IEEE divisions (scale, reciprocal, zero
// point) as before round 6's last trims
#ifndef AWQ_F16_PARAMS_FAST
#define AWQ_F16_PARAMS_FAST 1
#endif
struct FmtF16 {
    static constexpr int NW = 1, kBytes = 2;
    static constexpr bool kWide = false;
    static constexpr int kNanS = 0x7C00;
    static constexpr uint32_t kNanU = 0xFC00u, kSign = 0x8000u, kOnes = 0xFFFFu;
    __device__ static void lane_max(const Chunk<1>& c, int& smax, uint32_t& umax) { lane_max16(c.w[0], smax, umax); }
    __device__ static uint32_t lane_cmax(const Chunk<1>& c) { return lane_cmax16(c.w[0]); }
    __device__ static float dec(uint32_t h) { return (float)__builtin_bit_cast(_Float16, (uint16_t)h); }
    __device__ static float lo(uint32_t w) { return dec(w & 0xFFFFu); }
    __device__ static float hi(uint32_t w) { return dec(w >> 16); }
    __device__ static float rn(float a) { return (float)(_Float16)a; }   // v_cvt_f16_f32: RNE
    // z as an fp16 round trip (exact: an integer <= 255): RN(t + z) of two fp16 values is
    // then narrowed by the compiler to one v_add_f16 (exact: a single RNE fp16 add)
    __device__ static float as_fmt(float z) { return (float)(_Float16)z; }
    __device__ static float dq_scale(float s) { return s; }   // already an fp16 value
    // RN(x / s) for a positive finite s: Markstein-corrected quotient, exact for all fp16
    // pairs (oracle/verify_recip.c f16m; the plain x * RN(1/s) misses 2 990 pairs)
    __device__ static float quot(float x, float s, float r) {
        // x * r written as fma(x, r, -0) (bitwise the same product, signed zeros included)
        // so that both uses of x fold the fp16 -> f32 conversion into v_fma_mix_f32
        const float q0 = __builtin_fmaf(x, r, opaque_s(-0.0f));
        const float e = __builtin_fmaf(-s, q0, x);
        // RN_f32 first, as verified: a fused fma -> f16 (v_fma_mixlo_f16) rounds once
        return rn(opaque(__builtin_fmaf(e, r, q0)));
    }
#if AWQ_F16_PARAMS_FAST
    // RN_f16(d / qr) == RN_f16(d * RN_f32(1/qr)) for every non-negative fp16 d, inf included, and
    // qr = 2^bits - 1 (oracle/verify_recip.c f16scale); d * (1/qr) folds to a multiply by a constant
    __device__ static float scale(float d, float qr) { return rn(opaque(rn(d)) * (1.0f / qr)); }
    __device__ static float lo_clamp() { return 0.0f; }                            // RN_f16(1e-10) = 0
    __device__ static float recip(float s) { return recip_f16(s); }
    // RN(x / s): the Markstein quotient (exact for every fp16 x and positive finite fp16 s,
    // verify_recip f16m, with r the IEEE reciprocal recip_f16 returns) — the IEEE division only
    // for s = 0 / inf / NaN, in a branch the wave skips when no lane needs it
    __device__ static float quot_any(float x, float s, float r) {
        if (__builtin_expect(!(s > 0.0f && s < __builtin_inff()), 0)) return rn(opaque(x) / s);
        return quot(x, s, r);
    }
#else
    __device__ static float scale(float d, float qr) { return rn(opaque(rn(d)) / qr); }   // IEEE division
    __device__ static float lo_clamp() { return 0.0f; }                            // RN_f16(1e-10) = 0
    __device__ static float recip(float s) { return 1.0f / s; }
    __device__ static float quot_any(float x, float s, float r) {
        (void)r;
        return rn(opaque(x) / s);
    }
#endif
    // s = 0 (constant group: the fp16 clamp min is 0), inf or NaN -> exact special path
    __device__ static bool fast(float r) { return r > 0.0f && r < __builtin_inff(); }
    // The plain RN_f16(RN_f32(x * RN_f32(1/s))) misses RN_f16(x / s) only for scales
    // s >= 14 (302 of the 31 743 positive finite fp16 values, all >= 14; exhaustive,
    // oracle/verify_recip.c f16s): a tile whose 16 scales are all < 14 (every realistic
    // weight group: 4-bit s = range/15) takes one multiply per element instead of the
    // Markstein quotient.  The barrier keeps the product rounded to f32 first (a fused
    // v_mad_mixlo_f16 would round once).
    static constexpr bool kHasPlain = true;
    __device__ static bool plain_ok(float s) { return s < 14.0f; }
    __device__ static float quot_plain(float x, float r) { return rn(opaque(x * r)); }
    __device__ static float elem(const Chunk<1>& c, int i) {
        const uint32_t w = c.w[0][i >> 1];
        return (i & 1) ? hi(w) : lo(w);
    }
};

// fp32 weights: every op is the IEEE fp32 op (no rounding to a narrower dtype), x / s is
// the IEEE division itself (the kernel stays memory-bound: 4 B per element against the
// 16-bit formats' 2), min/max on the raw 32-bit patterns.
struct FmtF32 {
    static constexpr int NW = 2, kBytes = 4;
    static constexpr bool kWide = true;    // t + 8 is not exact in fp32: sym shifts after rint
    static constexpr int kNanS = 0x7F800000;
    static constexpr uint32_t kNanU = 0xFF800000u, kSign = 0x80000000u, kOnes = 0xFFFFFFFFu;
    __device__ static void lane_max(const Chunk<2>& c, int& smax, uint32_t& umax) {
        int sm = (int)c.w[0].x;
        uint32_t um = c.w[0].x;
#pragma unroll
        for (int i = 1; i < 8; ++i) {
            const uint32_t w = c.w[i >> 2][i & 3];
            sm = max(sm, (int)w);
            um = max(um, w);
        }
        smax = sm;
        umax = um;
    }
    __device__ static uint32_t lane_cmax(const Chunk<2>& c) {
        uint32_t m = ~c.w[0].x;
#pragma unroll
        for (int i = 1; i < 8; ++i) m = max(m, ~(uint32_t)c.w[i >> 2][i & 3]);
        return m;
    }
    __device__ static float dec(uint32_t h) { return __uint_as_float(h); }
    __device__ static float rn(float a) { return a; }
    __device__ static float as_fmt(float z) { return z; }
    __device__ static float dq_scale(float s) { return (float)(_Float16)s; }
    __device__ static float quot(float x, float s, float r) {
        (void)r;
        return x / s;                                   // IEEE (-fhip-fp32-correctly-rounded-divide-sqrt)
    }
    __device__ static float scale(float d, float qr) { return d / qr; }
    __device__ static float lo_clamp() { return 1e-10f; }                            // RN_f32(1e-10)
    __device__ static float recip(float s) { return 1.0f / s; }
    __device__ static float quot_any(float x, float s, float r) { return quot(x, s, r); }
    // s = inf (r = 0) or NaN -> exact special path; every finite s >= 1e-10 is fast
    __device__ static bool fast(float r) { return r > 0.0f && r < __builtin_inff(); }
    static constexpr bool kHasPlain = false;
    __device__ static bool plain_ok(float s) { (void)s; return false; }
    __device__ static float quot_plain(float x, float r) { return x * r; }
    __device__ static float elem(const Chunk<2>& c, int i) {
        const uint32_t w = c.w[i >> 2][i & 3];
        return __uint_as_float(w);
    }
};

struct GroupParams {
    float r;   // RN_f32(1 / s)
    float z;   // zero point (integral float; NaN only in special groups)
    float s;   // scale (a value of the input dtype)
};

// awq.py:192-199 on one group from the raw-bits reductions: smax = signed max of the bit
// patterns (sign-extended), umax = unsigned max, umin = unsigned min (only valid when the
// group is single-signed).  Returns the (NaN-propagated, symmetric-folded) [mn, mx] the
// scale is taken from.
template <typename F, bool SYM>
__device__ __forceinline__ void group_range(int smax, uint32_t umax, uint32_t umin, float& mn_out, float& mx_out,
                                            bool& nan_out) {
    const uint32_t mx_bits = smax >= 0 ? (uint32_t)smax : umin;   // all negative: smallest magnitude
    const uint32_t mn_bits = umax >= F::kSign ? umax : umin;      // none negative: smallest value
    const bool nan = (smax > F::kNanS) || (umax > F::kNanU);
    float mx = F::dec(mx_bits), mn = F::dec(mn_bits);
    if (nan) { mx = __builtin_nanf(""); mn = mx; }   // torch min/max both propagate NaN
    if (SYM) {                                        // awq.py:196-199
        float a = __builtin_fmaxf(__builtin_fabsf(mn), __builtin_fabsf(mx));
        if (nan) a = mx;
        mn = -a;
        mx = a;
    }
    mn_out = mn;
    mx_out = mx;
    nan_out = nan;
}

// awq.py:202-211: scale, reciprocal and zero point from the group's [mn, mx].
template <typename F, int BITS, bool SYM>
__device__ __forceinline__ GroupParams params_from_range(float mn, float mx) {
    constexpr float QR = (float)((1 << BITS) - 1);
    float s = F::scale(mx - mn, QR);                  // awq.py:202
    if (!__builtin_isnan(s)) s = __builtin_fmaxf(s, F::lo_clamp());   // awq.py:205
    GroupParams p;
    p.s = s;
    p.r = F::recip(s);
    if (SYM) {
        p.z = 0.0f;                                   // awq.py:208
    } else {
        const float y = F::quot_any(mn, s, p.r);      // RN(mn / s)
        float z = __builtin_rintf(-y);                // awq.py:210-211 (qmin = 0)
        if (!__builtin_isnan(z)) z = __builtin_fminf(__builtin_fmaxf(z, 0.0f), QR);
        p.z = z;
    }
    return p;
}

// The 8 fields of a lane packed from their unrounded values u: v_cvt_pk_u8_f32 rounds to
// nearest even and saturates to [0, 255] (scripts/cvt_probe.hip, every tie and edge on
// gfx950), so an 8-bit field is ONE conversion of u (= clamp(rint(u), 0, 255), the
// reference's round + clamp for qmin = 0 and, sym, for the field q + 128); a 4-bit field
// is a v_med3 clamp to [0, 15] then the conversion (rint(clamp(u)) == clamp(rint(u)) for
// integer bounds), the even elements' bytes OR-ed with the odd elements' shifted by 4.
template <int BITS>
__device__ __forceinline__ void pack8_cvt(const float (&u)[8], uint32_t& w0, uint32_t& w1) {
    if (BITS == 4) {
        uint32_t a = 0, b = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            a = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_amdgcn_fmed3f(u[2 * i], 0.0f, 15.0f), i, a);
            b = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_amdgcn_fmed3f(u[2 * i + 1], 0.0f, 15.0f), i, b);
        }
        w0 = a | (b << 4);
        w1 = 0;
    } else {
        uint32_t a = 0, b = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            a = __builtin_amdgcn_cvt_pk_u8_f32(u[i], i, a);
            b = __builtin_amdgcn_cvt_pk_u8_f32(u[4 + i], i, b);
        }
        w0 = a;
        w1 = b;
    }
}

// fp16 weights whose scales are all < 14 (the plain quotient, FmtF16::plain_ok): the field
// chain on packed f16 pairs (round 4).  t = RN_f16(x * r) is one v_cvt_pk_f16_f32 (RNE) per
// pair of f32 products, u = RN_f16(t + z) one v_pk_add_f16 — the reference's two roundings
// in the input dtype (awq.py:245-248) — then the clamp (v_pk_max / min_f16) and the round to
// an integer by adding 1024: at 2^10 the f16 ulp is 1, so the sum's RNE is 1024 + rint(u)
// and the half's bits are 0x6400 + field (rint(clamp(u)) == clamp(rint(u)) for integer
// bounds; 1024 + 255 < 2048 covers 8 bits).  Symmetric: clamp(t, -HALF, HALF - 1) + 1024 +
// HALF, whose RNE is 1024 + HALF + rint(t) (an even integer offset keeps ties to even) —
// the field rint(t) + HALF.  No NaN or inf reaches here (such groups are special).  The
// fields' low bytes are gathered by v_perm_b32 and, at 4 bits, folded into nibbles: ≈35
// VALU per 8 elements against ≈64 for the per-element f32 chain + v_cvt_pk_u8_f32.
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
template <int BITS, bool SYM>
__device__ __forceinline__ void pack8_f16_plain(const uint32_t (&d)[4], const float (&r)[8], const float (&z)[8],
                                                uint32_t& w0, uint32_t& w1) {
    constexpr _Float16 HALF = (_Float16)(1 << (BITS - 1));
    constexpr _Float16 QMAX = (_Float16)((1 << BITS) - 1);
    uint32_t P[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float x0 = (float)__builtin_bit_cast(_Float16, (uint16_t)(d[i] & 0xFFFFu));
        const float x1 = (float)__builtin_bit_cast(_Float16, (uint16_t)(d[i] >> 16));
        const float p0 = opaque(x0 * r[2 * i]), p1 = opaque(x1 * r[2 * i + 1]);   // f32 products
        const h2v t = __builtin_convertvector((f2){p0, p1}, h2v);                  // RN_f16 (RNE)
        h2v u;
        if (SYM) {
            u = __builtin_elementwise_min(__builtin_elementwise_max(t, (h2v){-HALF, -HALF}),
                                          (h2v){HALF - (_Float16)1, HALF - (_Float16)1});
            u = u + (h2v){(_Float16)1024 + HALF, (_Float16)1024 + HALF};
        } else {
            u = t + (h2v){(_Float16)z[2 * i], (_Float16)z[2 * i + 1]};             // RN_f16(t + z)
            u = __builtin_elementwise_min(__builtin_elementwise_max(u, (h2v){0, 0}), (h2v){QMAX, QMAX});
            u = u + (h2v){(_Float16)1024, (_Float16)1024};
        }
        P[i] = __builtin_bit_cast(uint32_t, u);
    }
    // bytes [q0 q1 q2 q3], [q4 q5 q6 q7] (each half's low byte)
    const uint32_t G0 = __builtin_amdgcn_perm(P[1], P[0], 0x06040200u);
    const uint32_t G1 = __builtin_amdgcn_perm(P[3], P[2], 0x06040200u);
    if (BITS == 8) {
        w0 = G0;
        w1 = G1;
    } else {
        const uint32_t t0 = G0 | (G0 >> 4), t1 = G1 | (G1 >> 4);   // bytes 0 / 2: q0 | q1 << 4, ...
        w0 = __builtin_amdgcn_perm(t1, t0, 0x06040200u);
        w1 = 0;
    }
}

// Quantize the 8 values of one lane (awq.py:245-248) for a group with a positive finite
// scale and pack them: 4-bit -> w.x, 8-bit -> (w.x, w.y).  Field value = q - qmin.
template <typename F, int BITS, bool SYM, bool PLAIN = false>
__device__ __forceinline__ u2v quant8_fast(const Chunk<F::NW>& v, float r, float z, float s) {
    if constexpr (std::is_same<F, FmtF16>::value && PLAIN) {
        const uint32_t d[4] = {v.w[0].x, v.w[0].y, v.w[0].z, v.w[0].w};
        const float rr[8] = {r, r, r, r, r, r, r, r}, zz[8] = {z, z, z, z, z, z, z, z};
        uint32_t w0, w1;
        pack8_f16_plain<BITS, SYM>(d, rr, zz, w0, w1);
        u2v w;
        w.x = w0;
        w.y = w1;
        return w;
    }
    constexpr float HALF = (float)(1 << (BITS - 1));
    const float zf = F::as_fmt(z);
    float q[8];   // the field before rounding: clamp + RNE are the pack's v_cvt_pk_u8_f32
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        // RN(x / s)
        const float x0 = F::elem(v, 2 * i), x1 = F::elem(v, 2 * i + 1);
        const float t0 = PLAIN ? F::quot_plain(x0, r) : F::quot(x0, s, r);
        const float t1 = PLAIN ? F::quot_plain(x1, r) : F::quot(x1, s, r);
        float u0, u1;
        if (SYM && F::kWide) {
            u0 = __builtin_rintf(t0) + HALF;                         // exact: an integer + 8
            u1 = __builtin_rintf(t1) + HALF;
        } else if (SYM) {
            u0 = t0 + HALF;                                          // rint(t)+8 == rint(t+8)
            u1 = t1 + HALF;                                          // (exact for 16-bit t)
        } else {
            u0 = F::rn(t0 + zf);                                     // RN(x/s + z)
            u1 = F::rn(t1 + zf);
        }
        q[2 * i] = u0;
        q[2 * i + 1] = u1;
    }
    uint32_t w0, w1;
    pack8_cvt<BITS>(q, w0, w1);
    u2v w;
    w.x = w0;
    w.y = w1;
    return w;
}


// Same with the reference's NaN/inf semantics (groups whose scale is 0, inf or NaN), with
// a true IEEE division per element.
template <typename F, int BITS, bool SYM>
__device__ __forceinline__ void quant8_special(const Chunk<F::NW>& v, float z, float s, uint32_t (&nib)[8],
                                               int32_t (&q)[8]) {
    constexpr int QMIN = SYM ? -(1 << (BITS - 1)) : 0;
    constexpr int QMAX = SYM ? (1 << (BITS - 1)) - 1 : (1 << BITS) - 1;
    constexpr uint32_t MASK = (1u << BITS) - 1u;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const float x = F::elem(v, i);
        const float t = F::rn(opaque(x) / s);
        const float u = SYM ? t : F::rn(t + z);
        float rr = __builtin_rintf(u);
        int32_t qi;
        if (__builtin_isnan(rr)) {
            qi = INT32_MIN;
        } else {
            rr = __builtin_fminf(__builtin_fmaxf(rr, (float)QMIN), (float)QMAX);
            qi = (int32_t)rr;
        }
        q[i] = qi;
        nib[i] = ((uint32_t)qi - (uint32_t)QMIN) & MASK;
    }
}

// fp16 bits of a group's scale (awq.py:411); NaN scales per nan_scale_code (awq_internal.h):
// gnan = the group holds a NaN (else the NaN came from inf - inf)
__device__ __forceinline__ uint16_t f16_bits(float s, bool gnan, uint32_t nan_code) {
    if (__builtin_isnan(s)) return nan_scale_pick(nan_code, gnan);
    _Float16 h = (_Float16)s;                          // v_cvt_f16_f32: RNE, subnormals kept
    return __builtin_bit_cast(uint16_t, h);
}

// ---------------------------------------------------------------------------------------
// Tile context: everything a wave needs about one tile, all wave-uniform (SGPRs).
// ---------------------------------------------------------------------------------------

}  // namespace
}  // namespace awq
#endif  // AWQ_QUANT_H
