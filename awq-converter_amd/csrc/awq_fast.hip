// awq_fast.hip — streaming group quantizer for bf16 / fp16 / fp32 weights, group_size
// 32, 64, 128 or 256 (gfx950).
//
// Replaces the per-group Python double loop of the reference
// (src/awq_quantizer/quantization/awq.py:286-374 -> _compute_scale_zp_for_group :173-213
// -> _quantize_tensor :215-250) with one HBM pass: read the weights once, write packed
// qweight/qzeros + fp16 scales (and, in parity mode, the reference's unpacked int32
// tensor_q / zero_points).
//
// Mapping (HBM-bound, no MFMA; described for bf16, GS 128 — the benchmark — with the
// general rule in brackets):
//   * one wave = one tile = 2048 elements = 4 KiB of bf16 [2048 / GS group slots]; lane l
//     holds elements 512 j + 8 l .. + 7 of load j, one 16-B buffer_load_dwordx4 [two for
//     fp32], so a group spans 16 lanes [L = GS / 8] and lane-row rho holds groups 4j + rho;
//   * the grid has one wave per tile (non-persistent): the hardware dispatcher hands a
//     finished wave's slot to the next workgroup, which balances the load across CUs.  A
//     persistent grid (waves walking tiles) lost ~20 % to the dispatcher's age priority:
//     the youngest workgroups of every CU ran last and alone (profiles/r24-r27);
//   * per-group min/max from the raw bits (signed / unsigned integer max), reduced over
//     the group's lanes with DPP-fused v_max [plus one v_permlane16_swap at GS 256]; NaN
//     is detected from the bits;
//   * the scale / zero point of the tile's groups are computed ONCE per lane set (lane c of
//     a group owns the group of load c & 3), with the reference's per-op rounding, then
//     broadcast to the group's lanes with one DPP quad_perm per parameter;
//   * per element: RN_bf16(x * RN_f32(1/s)) == RN_bf16(x / s) for every bf16 x and every
//     bf16 s >= RN_bf16(1e-10) (verified exhaustively: oracle/verify_recip.c), so one
//     multiply replaces the division; RNE to bf16 is one v_cvt_pk_bf16_f32 with a zero
//     low half (the dword IS the rounded f32); + z, round-half-even, clamp, and
//     v_cvt_pk_u8_f32 packs nibble pairs / bytes [fp16: plain or Markstein quotient;
//     fp32: the IEEE division];
//   * each lane emits one packed int32 per load (4-bit), staged in LDS into one 16-B store
//     per lane;
//   * buffer descriptors are based at the tile start with the tile's byte length, so
//     slots past the tile end read zeros and their stores are dropped by the hardware
//     range check (no per-lane masks, no OOB access, tensors > 4 GB are fine).
// Ragged launches: one grid over the tiles of many tensors (descriptor table in HBM); a
// wave finds its tensor from a host-planned per-workgroup table (or, without it, a
// 64-lane ballot search of the descriptors).
#include <cstdlib>
#include <type_traits>

#include "awq_internal.h"

// Build-time knobs (scripts/kbench.py compares variants; defaults measured best).
// cache-policy bits of the input loads and the qweight / tensor_q stores (gfx950: 2 = nt)
#ifndef AWQ_LOAD_AUX
#define AWQ_LOAD_AUX 2
#endif
#ifndef AWQ_STORE_AUX
#define AWQ_STORE_AUX 2
#endif
// cache policy of the small per-tile stores (scales, zeros, qzeros: 8-32 B per tile).
// Default policy (0), not nt: the L2 then merges the partial lines neighbouring tiles
// write (measured +2-5 % over nt, profiles/r19-r20)
#ifndef AWQ_SMALL_AUX
#define AWQ_SMALL_AUX 0
#endif
// __launch_bounds__ minimum waves per SIMD (8 = 32 waves per CU: <= 64 VGPRs, <= 80 SGPRs)
#ifndef AWQ_MIN_WAVES
#define AWQ_MIN_WAVES 8
#endif
// same for fp32 inputs (32 data VGPRs per lane instead of 16)
#ifndef AWQ_MIN_WAVES_WIDE
#define AWQ_MIN_WAVES_WIDE 6
#endif
// qweight stores: 1 = staged through LDS into one 16-B store per lane (4-bit: 1 store
// instruction per tile instead of 4), 0 = one dword per lane per group row
#ifndef AWQ_WIDE_STORE
#define AWQ_WIDE_STORE 1
#endif

#ifndef AWQ_F16_PLAIN
#define AWQ_F16_PLAIN 1
#endif
// XCD runs: consecutive workgroups are dealt round-robin over the 8 XCDs (each with its
// own L2), so with one-wave workgroups neighbouring tiles — which share the 128-B lines of
// the scales (32 B per tile) and qzeros (8 B per tile) outputs — would write those lines
// partially from different L2s.  Remapping block b so every XCD takes runs of
// AWQ_XCD_RUN consecutive blocks keeps each line's writers on one L2 (0 = no remap)
#ifndef AWQ_XCD_RUN
#define AWQ_XCD_RUN 0
#endif

namespace awq {
namespace {

typedef short s2 __attribute__((ext_vector_type(2)));
typedef unsigned short us2 __attribute__((ext_vector_type(2)));
typedef float f2 __attribute__((ext_vector_type(2)));
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

// RN_f32(1/s) for a bf16-valued s: v_rcp_f32 + one Newton step with fma is correctly
// rounded for every bf16 s < 2^126 (checked exhaustively on the GPU by awq_selftest);
// larger, inf and NaN go through the IEEE division.
__device__ __forceinline__ float recip_bf16(float s) {
    if (__builtin_expect(!(s < 0x1p126f), 0)) return 1.0f / s;
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
    __device__ static float scale(float d, float qr) { return rn(opaque(rn(d)) / qr); }   // IEEE division
    __device__ static float lo_clamp() { return 0.0f; }                            // RN_f16(1e-10) = 0
    __device__ static float recip(float s) { return 1.0f / s; }
    __device__ static float quot_any(float x, float s, float r) {
        (void)r;
        return rn(opaque(x) / s);
    }
    // s = 0 (constant group: the fp16 clamp min is 0), inf or NaN -> exact special path
    __device__ static bool fast(float r) { return r > 0.0f && r < __builtin_inff(); }
    // The plain RN_f16(RN_f32(x * RN_f32(1/s))) misses RN_f16(x / s) only for scales
    // s >= 14 (302 of the 31 743 positive finite fp16 values, all >= 14; exhaustive,
    // oracle/verify_recip.c f16s): a tile whose 16 scales are all < 14 (every realistic
    // weight group: 4-bit s = range/15) takes one multiply per element instead of the
    // Markstein quotient.  The barrier keeps the product rounded to f32 first (a fused
    // v_mad_mixlo_f16 would round once).
    static constexpr bool kHasPlain = AWQ_F16_PLAIN;   // tuning builds: -DAWQ_F16_PLAIN=0
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

// Quantize the 8 values of one lane (awq.py:245-248) for a group with a positive finite
// scale and pack them: 4-bit -> w.x, 8-bit -> (w.x, w.y).  Field value = q - qmin.
template <typename F, int BITS, bool SYM, bool PLAIN = false>
__device__ __forceinline__ u2v quant8_fast(const Chunk<F::NW>& v, float r, float z, float s) {
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
struct TileCtx {
    int32_t* qweight;    // tensor bases of the outputs (nullptr = not wanted)
    int32_t* qzeros;
    uint16_t* scales;
    int32_t* tensor_q;
    int32_t* zeros;
    uint32_t start;      // flat group index of the tile's first group
    uint32_t ng;         // groups in the tile (<= S = 2048 / GS)
    uint32_t w0, nw;     // qzeros word range
    uint32_t G, WPR;     // geometry (see awq_internal.h)
    uint32_t r0, g0;     // row / group-in-row of the tile's first group
    uint32_t bytes;      // byte tiles (qzeros written byte-wise) vs word tiles
    uint64_t el_off;     // first input / tensor_q element of the tile
    uint32_t valid;      // elements of the tile inside the tensor (padded rows: inside the row)
    uint64_t qw_off;     // first qweight word of the tile
    uint32_t qw_n;       // qweight words of the tile
};

template <int BITS, int GS, bool PAD>
__device__ __forceinline__ TileCtx make_ctx(const awq_tensor_desc& d, uint32_t tile) {
    constexpr uint32_t S = kTileElems / GS;
    const TensorGeom g = fast_geom(d.rows, d.K, BITS, GS, PAD);
    constexpr uint32_t WPG = GS * BITS / 32;   // qweight words per group
    TileCtx c;
    c.bytes = g.bytes;
    if (g.TR) {                                // padded rows: row tiles
        const uint32_t r = tile / g.TR;
        c.r0 = r;
        c.g0 = (tile - r * g.TR) * S;
        c.ng = min(S, g.G - c.g0);
        c.start = r * g.G + c.g0;
        c.w0 = r * g.WPR + c.g0 / g.C;
        c.nw = (c.ng + g.C - 1) / g.C;
        c.el_off = (uint64_t)r * (uint64_t)d.K + (uint64_t)c.g0 * GS;
        c.valid = (uint32_t)min((int64_t)c.ng * GS, d.K - (int64_t)c.g0 * GS);
        c.qw_off = (uint64_t)r * (uint64_t)(d.K * BITS / 32) + (uint64_t)c.g0 * WPG;
        c.qw_n = c.valid * BITS / 32;
    } else if (g.bytes) {
        c.start = tile * S;
        c.ng = min(S, (uint32_t)d.rows * g.G - c.start);
        c.r0 = c.start / g.G;
        c.g0 = c.start - c.r0 * g.G;
        c.w0 = 0;
        c.nw = 0;
    } else {
        const uint32_t w0 = tile * g.WPT;
        const uint32_t w1 = min(w0 + g.WPT, g.words);
        const uint32_t r0 = w0 / g.WPR;
        c.r0 = r0;
        c.g0 = (w0 - r0 * g.WPR) * g.C;
        c.start = r0 * g.G + c.g0;
        const uint32_t end = (w1 == g.words) ? (uint32_t)d.rows * g.G : word_group(g, w1);
        c.ng = end - c.start;
        c.w0 = w0;
        c.nw = w1 - w0;
    }
    if (!g.TR) {
        c.el_off = (uint64_t)c.start * GS;
        c.valid = c.ng * GS;
        c.qw_off = (uint64_t)c.start * WPG;
        c.qw_n = c.ng * WPG;
    }
    c.G = g.G;
    c.WPR = g.WPR;
    c.qweight = d.qweight;
    c.qzeros = d.qzeros;
    c.scales = d.scales;
    c.tensor_q = d.tensor_q;
    c.zeros = d.zeros;
    return c;
}

// first element and element count of a tile (the input range it reads; padded rows stop at
// the row end, the range check supplies the zero padding)
template <int BITS, int GS, bool PAD>
__device__ __forceinline__ void tile_src(int64_t rows, int64_t K, uint32_t tile, uint64_t& el_off, uint32_t& valid) {
    constexpr uint32_t S = kTileElems / GS;
    const TensorGeom g = fast_geom(rows, K, BITS, GS, PAD);
    if (g.TR) {
        const uint32_t r = tile / g.TR;
        const uint32_t g0 = (tile - r * g.TR) * S;
        el_off = (uint64_t)r * (uint64_t)K + (uint64_t)g0 * GS;
        valid = (uint32_t)min((int64_t)S * GS, K - (int64_t)g0 * GS);
        return;
    }
    uint32_t start, ng;
    if (g.bytes) {
        start = tile * S;
        ng = min(S, (uint32_t)rows * g.G - start);
    } else {
        const uint32_t w0 = tile * g.WPT;
        const uint32_t w1 = min(w0 + g.WPT, g.words);
        start = word_group(g, w0);
        const uint32_t end = (w1 == g.words) ? (uint32_t)rows * g.G : word_group(g, w1);
        ng = end - start;
    }
    el_off = (uint64_t)start * GS;
    valid = ng * GS;
}

// 4 x 16-B loads per lane: load j covers the tile's bytes [1 KiB j, 1 KiB (j+1)), lane l
// its 16 B at 16 l — group slot j * (64 / L) + l / L, chunk l % L of that group
// (L = GS / 8).  Slots past the tile end fall outside the descriptor's range and read as
// zero.
// fp32: the same element mapping, each lane's 32 B as two 16-B loads (a pair of
// instructions covers 2 KiB contiguously).
template <typename F, int GS>
__device__ __forceinline__ void load_tile(const char* wp, uint32_t valid, Chunk<F::NW> (&v)[4]) {
    const int lane = threadIdx.x & 63;
    const __amdgpu_buffer_rsrc_t rw = rsrc(wp, valid * (uint32_t)F::kBytes);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int h = 0; h < F::NW; ++h)
            v[j].w[h] = __builtin_amdgcn_raw_buffer_load_b128(
                rw, (uint32_t)(j * 512 * F::kBytes + lane * 8 * F::kBytes + 16 * h), 0, AWQ_LOAD_AUX);
}

// sum over the L lanes of a group, pairwise over adjacent lanes (xor 1, xor 2, then the
// half-row and row mirrors and the row swap pair adjacent blocks): every lane ends with the
// same value, the tree include/awq_hip.h (awq_quantize_search) defines for the clip-search
// error
template <int CTRL>
__device__ __forceinline__ float dpp_add(float v) {
    return v + __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
template <int L>
__device__ __forceinline__ float grp_sum(float v) {
    v = dpp_add<0xB1>(v);                  // quad_perm [1,0,3,2]
    v = dpp_add<0x4E>(v);                  // quad_perm [2,3,0,1]
    if (L >= 8) v = dpp_add<0x141>(v);     // row_half_mirror
    if (L >= 16) v = dpp_add<0x140>(v);    // row_mirror
    if (L >= 32) {                         // (row 2k) + (row 2k+1) on both rows
        const auto p = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v),
                                                        false, false);
        v = __builtin_bit_cast(float, (unsigned)p[0]) + __builtin_bit_cast(float, (unsigned)p[1]);
    }
    return v;
}

// Squared error of this lane's 8-element chunk of a group for one candidate (r, z, s) —
// quantize (awq.py:245-248), dequantize the reference's way (fp16(fp16(q - z) * fp16(s)),
// awq.py:459-539), (x - dq)^2 summed in element order.  `special`: the candidate's scale
// is 0 / inf / NaN (exact division, NaN-propagating clamp).
template <typename F, int BITS, bool SYM>
__device__ __forceinline__ float chunk_err(const Chunk<F::NW>& v, float r, float z, float s, float sh, bool special) {
    constexpr float QMIN = SYM ? -(float)(1 << (BITS - 1)) : 0.0f;
    constexpr float QMAX = SYM ? (float)((1 << (BITS - 1)) - 1) : (float)((1 << BITS) - 1);
    const float zf = F::as_fmt(z);
    float acc = 0.0f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const float x = F::elem(v, i);
        float q;
        if (__builtin_expect(special, 0)) {
            const float t = F::rn(opaque(x) / s);
            const float rr = __builtin_rintf(SYM ? t : F::rn(t + zf));
            q = __builtin_isnan(rr) ? rr : __builtin_fminf(__builtin_fmaxf(rr, QMIN), QMAX);
        } else {
            const float t = F::quot(x, s, r);
            q = __builtin_fminf(__builtin_fmaxf(__builtin_rintf(SYM ? t : F::rn(t + zf)), QMIN), QMAX);
        }
        const float dq = (float)(_Float16)((q - zf) * sh);
        const float d = x - dq;
        acc = acc + d * d;
    }
    return acc;
}

// Opt-in clip search (include/awq_hip.h awq_quantize_search) inside the streaming kernel:
// candidates alpha_i = (n_grid - i) / n_grid shrink [mn, mx]; lane (grp, ch) evaluates the
// candidate's parameters for its parameter group (the one in load ch & 3), the L lanes of a
// group score each of its 4 loads' groups (8 elements per lane, grp_sum), and the smallest
// error (ties: the earlier candidate; NaN never wins) picks the group's final [mn, mx].
// RN(v * alpha) as torch evaluates it (fp32 product, then one rounding to the dtype); the
// barrier stops the fp16 product from becoming a single-rounding v_mad_mixlo_f16
template <typename F>
__device__ __forceinline__ float shrink(float v, float al) {
    return F::rn(opaque(v * al));
}

template <typename F, int BITS, bool SYM, int GS>
__device__ __forceinline__ void search_range(const Chunk<F::NW> (&v)[4], float& gmn, float& gmx, bool gnan, int n_grid,
                                          int n_cand) {
    const int jj = threadIdx.x & 3;
    float best = __builtin_inff();
    int bi = 0;
    for (int i = 0; i < n_cand; ++i) {
        const float al = (float)(n_grid - i) / (float)n_grid;
        const GroupParams cp = params_from_range<F, BITS, SYM>(shrink<F>(gmn, al), shrink<F>(gmx, al));
        const float csh = F::dq_scale(cp.s);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float rj = bcast_j(j, cp.r);
            const float zj = SYM ? 0.0f : bcast_j(j, cp.z);
            const float sj = bcast_j(j, cp.s);
            const float hj = bcast_j(j, csh);
            const bool special = !F::fast(rj);
            float e;
            if (__builtin_expect(__ballot(special) != 0, 0)) e = chunk_err<F, BITS, SYM>(v[j], rj, zj, sj, hj, special);
            else e = chunk_err<F, BITS, SYM>(v[j], rj, zj, sj, hj, false);
            e = grp_sum<GS / 8>(e);
            if (j == jj && e < best) {
                best = e;
                bi = i;
            }
        }
    }
    if (!gnan && bi != 0) {
        const float al = (float)(n_grid - bi) / (float)n_grid;
        gmn = shrink<F>(gmn, al);
        gmx = shrink<F>(gmx, al);
    }
}

template <typename F, int BITS, bool SYM, bool SEARCH, int GS>
__device__ __forceinline__ void compute_tile(const TileCtx& c, const Chunk<F::NW> (&v)[4], uint32_t* zw, uint32_t* qstage,
                                             int n_grid, int n_cand, uint32_t nan_code) {
    constexpr int QMIN = SYM ? -(1 << (BITS - 1)) : 0;
    constexpr uint32_t C = 32u / BITS;   // groups per qzeros word
    constexpr int L = GS / 8;            // lanes per group (8 elements = 16 B per lane)
    constexpr int GPJ = 64 / L;          // groups per load instruction
    constexpr uint32_t S = 4 * GPJ;      // group slots per tile
    const int lane = threadIdx.x & 63;
    const int grp = lane / L;            // group of this lane inside each load
    const int ch = lane % L;             // 16-B chunk of the group
    const uint32_t ng = c.ng;
#ifdef AWQ_TRIVIAL_COMPUTE
    // timing-only build (scripts/kbench.py): same loads and stores, no arithmetic
    if (c.qweight) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t word = v[j].w[0].x ^ v[j].w[0].y ^ v[j].w[0].z ^ v[j].w[F::NW - 1].w;
            __amdgpu_buffer_rsrc_t rq = rsrc(c.qweight + c.qw_off, c.qw_n * 4u);
            __builtin_amdgcn_raw_buffer_store_b32(word, rq, (uint32_t)((64 * j + lane) * 4), 0, AWQ_STORE_AUX);
        }
    }
#ifndef AWQ_TRIVIAL_NOSMALL
    if (ch < 4 && c.scales) {
        __amdgpu_buffer_rsrc_t rs = rsrc(c.scales + c.start, ng * 2u);
        __builtin_amdgcn_raw_buffer_store_b16((uint16_t)v[0].w[0].x, rs, (GPJ * ch + grp) * 2u, 0, AWQ_SMALL_AUX);
    }
    if (c.qzeros && (uint32_t)lane < c.nw) {
        __amdgpu_buffer_rsrc_t rz = rsrc(c.qzeros + c.w0, c.nw * 4u);
        __builtin_amdgcn_raw_buffer_store_b32(v[1].w[0].y, rz, (uint32_t)lane * 4u, 0, AWQ_SMALL_AUX);
    }
#endif
    return;
#endif

    // ---- 1. group min/max (awq.py:192-193) of the 4 groups this lane's group-lanes hold,
    //         from the raw 16-bit patterns: the SIGNED int16 max is the float max whenever
    //         the group has a value with the sign bit clear, and the UNSIGNED max is the
    //         float min (most negative) whenever it has one with the sign bit set; NaNs land
    //         beyond F::kNanS / F::kNanU.  Single-signed groups (rare in weights; LayerNorm
    //         gammas) take an extra unsigned-min reduction in a wave-uniform branch.
    //         Reductions over the group's L lanes: DPP-fused v_max_i32 (grp_max) ----
    int smx[4];
    uint32_t umx[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        int sm;
        uint32_t um;
        F::lane_max(v[j], sm, um);
        smx[j] = grp_max<L>(sm);
        umx[j] = grp_max<L>(um);
    }
    uint32_t umn[4] = {0, 0, 0, 0};
    bool one_signed = false;
#pragma unroll
    for (int j = 0; j < 4; ++j) one_signed |= (smx[j] < 0) || (umx[j] < F::kSign);
    if (__builtin_expect(__ballot(one_signed) != 0, 0)) {
#pragma unroll
        for (int j = 0; j < 4; ++j) umn[j] = F::kOnes - grp_max<L>(F::lane_cmax(v[j]));   // unsigned min
    }
    // ---- 2. scale / zero point: lane (grp, ch) computes the group of load ch & 3, i.e.
    //         slot GPJ * (ch & 3) + grp (the L / 4 lanes of a group with equal ch & 3 do the
    //         same work; for GS 32 every lane owns exactly one of the 64 slots) ----
    const int jj = ch & 3;
    int ssel = smx[0];
    uint32_t usel = umx[0], nsel = umn[0];
#pragma unroll
    for (int j = 1; j < 4; ++j)
        if (jj == j) { ssel = smx[j]; usel = umx[j]; nsel = umn[j]; }
    float gmn, gmx;
    bool gnan;
    group_range<F, SYM>(ssel, usel, nsel, gmn, gmx, gnan);
    if (SEARCH && n_cand > 1) search_range<F, BITS, SYM, GS>(v, gmn, gmx, gnan, n_grid, n_cand);
    const GroupParams p = params_from_range<F, BITS, SYM>(gmn, gmx);
    const uint32_t my_slot = GPJ * (uint32_t)jj + (uint32_t)grp;
    // wave-uniform: every group of the tile admits the plain quotient (F::plain_ok)
    const bool plain = F::kHasPlain && __builtin_amdgcn_ballot_w64(!F::plain_ok(p.s)) == 0;

    // ---- 4. quantize + pack the 4 groups of this lane ----
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        // this group's r, z, s from the quad lane with ch & 3 == j, broadcast just in time
        // (short live ranges)
        const float rj = bcast_j(j, p.r);
        const float zj = SYM ? 0.0f : bcast_j(j, p.z);
        const float sj = bcast_j(j, p.s);
        u2v word = plain ? quant8_fast<F, BITS, SYM, true>(v[j], rj, zj, sj)
                         : quant8_fast<F, BITS, SYM, false>(v[j], rj, zj, sj);
        const bool special = !F::fast(rj);         // scale 0 / inf / NaN
        if (__builtin_expect(special, 0)) {
            // (q values stay local to the rare branches: a q array live across them made
            // the compiler zero-initialise 8 registers per j on the common path)
            uint32_t nib[8];
            int32_t qs[8];
            quant8_special<F, BITS, SYM>(v[j], zj, sj, nib, qs);
            if (BITS == 4) {
                uint32_t acc = 0;
#pragma unroll
                for (int i = 0; i < 8; ++i) acc |= nib[i] << (4 * i);
                word.x = acc;
            } else {
                word.x = nib[0] | (nib[1] << 8) | (nib[2] << 16) | (nib[3] << 24);
                word.y = nib[4] | (nib[5] << 8) | (nib[6] << 16) | (nib[7] << 24);
            }
        }
        // this lane's 8 elements are tile elements 512 j + 8 lane: packed word 64 j + lane
        if (c.qweight) {
#if AWQ_WIDE_STORE
            // staged in the wave's LDS block in output order (the lanes of one j write 64
            // consecutive words), stored below as one 16-B piece per lane
            if (BITS == 4) qstage[64 * j + lane] = word.x;
            else *(u2v*)(qstage + 128 * j + 2 * lane) = word;
#else
            __amdgpu_buffer_rsrc_t rq = rsrc(c.qweight + c.qw_off, c.qw_n * 4u);
            if (BITS == 4)
                __builtin_amdgcn_raw_buffer_store_b32(word.x, rq, (uint32_t)((64 * j + lane) * 4), 0, AWQ_STORE_AUX);
            else
                __builtin_amdgcn_raw_buffer_store_b64(word, rq, (uint32_t)((64 * j + lane) * 8), 0, AWQ_STORE_AUX);
#endif
        }
        if (c.tensor_q) {   // reference-layout int32 tensor_q (parity mode)
            int32_t q[8];
            if (__builtin_expect(special, 0)) {
                uint32_t nib[8];
                quant8_special<F, BITS, SYM>(v[j], zj, sj, nib, q);
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const uint32_t wd = (BITS == 4) ? word.x : (i < 4 ? word.x : word.y);
                    const uint32_t sh = (BITS == 4) ? 4 * i : 8 * (i & 3);
                    q[i] = (int32_t)((wd >> sh) & ((1u << BITS) - 1u)) + QMIN;
                }
            }
            __amdgpu_buffer_rsrc_t rt = rsrc(c.tensor_q + c.el_off, c.valid * 4u);
            u4 lo = {(uint32_t)q[0], (uint32_t)q[1], (uint32_t)q[2], (uint32_t)q[3]};
            u4 hi = {(uint32_t)q[4], (uint32_t)q[5], (uint32_t)q[6], (uint32_t)q[7]};
            __builtin_amdgcn_raw_buffer_store_b128(lo, rt, (uint32_t)((512 * j + 8 * lane) * 4), 0, AWQ_STORE_AUX);
            __builtin_amdgcn_raw_buffer_store_b128(hi, rt, (uint32_t)((512 * j + 8 * lane) * 4 + 16), 0, AWQ_STORE_AUX);
        }
    }
#if AWQ_WIDE_STORE
    if (c.qweight) {   // 4-bit: 1 KiB per tile = one dwordx4 per lane; 8-bit: 2 KiB, two
        __amdgpu_buffer_rsrc_t rq = rsrc(c.qweight + c.qw_off, c.qw_n * 4u);
#pragma unroll
        for (int h = 0; h < (BITS == 4 ? 1 : 2); ++h) {
            const u4 w4 = *(const u4*)(qstage + h * 256 + lane * 4);
            __builtin_amdgcn_raw_buffer_store_b128(w4, rq, (uint32_t)(h * 1024 + lane * 16), 0, AWQ_STORE_AUX);
        }
    }
#endif
    // ---- 5. per-group scalars out (after the data registers are dead): lanes ch < 4 hold
    //         the S slots (one store each) ----
    if (ch < 4) {
        if (c.scales) {
            __amdgpu_buffer_rsrc_t rs = rsrc(c.scales + c.start, ng * 2u);
            __builtin_amdgcn_raw_buffer_store_b16(f16_bits(p.s, gnan, nan_code), rs, my_slot * 2u, 0, AWQ_SMALL_AUX);
        }
        if (c.zeros) {
            __amdgpu_buffer_rsrc_t rz = rsrc(c.zeros + c.start, ng * 4u);
            int32_t zi = __builtin_isnan(p.z) ? INT32_MIN : (int32_t)p.z;
            __builtin_amdgcn_raw_buffer_store_b32((uint32_t)zi, rz, my_slot * 4u, 0, AWQ_SMALL_AUX);
        }
    }
    // qzeros, byte tiles: each group's field OR-ed into its byte (wave-private LDS), then one
    // lane per qzeros byte stores it (plus the zero pad bytes ending its row's last word)
    if (c.qzeros && c.bytes) {
        constexpr uint32_t GPB = BITS == 4 ? 2u : 1u;        // groups per byte
        if ((uint32_t)lane < S) zw[lane] = 0u;
        if (ch < 4 && my_slot < ng) {
            uint32_t zn = __builtin_isnan(p.z) ? (uint32_t)(0u - (uint32_t)QMIN) : (uint32_t)((int)p.z - QMIN);
            zn &= (1u << BITS) - 1u;
            atomicOr(&zw[my_slot / GPB], zn << (BITS * (my_slot % GPB)));
        }
        const uint32_t nb = ng / GPB;                         // ng and the tile start are even
        if ((uint32_t)lane < nb) {
            uint32_t g = c.g0 + (uint32_t)lane * GPB, r = c.r0;
            if (g >= c.G) {
                const uint32_t k = g / c.G;
                r += k;
                g -= k * c.G;
            }
            const uint32_t row_bytes = c.WPR * 4u;
            __amdgpu_buffer_rsrc_t rz = rsrc(c.qzeros, 0x7FFFFFFFu);
            const uint32_t at = r * row_bytes + g / GPB;
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)zw[lane], rz, at, 0, AWQ_SMALL_AUX);
            if (g + GPB >= c.G) {                               // row's last byte: zero the pad
                for (uint32_t b = g / GPB + 1; b < row_bytes; ++b)
                    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)0, rz, r * row_bytes + b, 0, AWQ_SMALL_AUX);
            }
        }
    }
    // qzeros, word tiles: each slot's field OR-ed into its word (wave-private LDS), then stored
    if (c.qzeros && !c.bytes) {
        if ((uint32_t)lane < S) zw[lane] = 0u;
        if (ch < 4 && my_slot < ng) {
            uint32_t g = c.g0 + my_slot, r = c.r0;
            if (g >= c.G) {                 // slot lies in a later row of the tile
                const uint32_t k = g / c.G;
                r += k;
                g -= k * c.G;
            }
            const uint32_t wi = r * c.WPR + g / C;
            const uint32_t pos = g % C;
            uint32_t zn = __builtin_isnan(p.z) ? (uint32_t)(0u - (uint32_t)QMIN) : (uint32_t)((int)p.z - QMIN);
            zn &= (1u << BITS) - 1u;
            atomicOr(&zw[wi - c.w0], zn << (BITS * pos));
        }
        if ((uint32_t)lane < c.nw) {
            __amdgpu_buffer_rsrc_t rz = rsrc(c.qzeros + c.w0, c.nw * 4u);
            __builtin_amdgcn_raw_buffer_store_b32(zw[lane], rz, (uint32_t)lane * 4u, 0, AWQ_SMALL_AUX);
        }
    }

}

// Bijective block renumbering for XCD runs (AWQ_XCD_RUN): block b, dealt to XCD b % 8,
// takes the (b / 8) % R-th block of XCD b % 8's run inside super-chunk b / (8 R); blocks of
// the last, partial super-chunk keep their index.
__device__ __forceinline__ int64_t xcd_run_block(int64_t b, int64_t nblocks) {
    constexpr int64_t R = AWQ_XCD_RUN > 0 ? AWQ_XCD_RUN : 1, X = 8;   // (only called when AWQ_XCD_RUN > 0)
    const int64_t full = nblocks / (X * R) * (X * R);
    if (b >= full) return b;
    const int64_t x = b % X, i = b / X;
    return (i / R) * (X * R) + x * R + (i % R);
}

// ---------------------------------------------------------------------------------------
// Any group size up to 512 (bf16 / fp16; 256 for fp32), any K: row-segment tiles.
//
// A tile = GPT consecutive groups of one row (GPT a multiple of 8 up to 64; the cost model
// picks 8, 16, 32 or 64), one 64-lane wave per tile:
//   stage   the segment's bytes go to LDS with 16-B loads, all in flight at once (16-B
//           aligned start; the tensor's last bytes go by 2-B loads);
//   pass 1  lane (grp, j) owns chunk j of group grp (P lanes per group = the largest power
//           of two <= 64 / the tile's groups, C = ceil(L / P) elements each) and reduces
//           the raw-bits min/max over it (packed 16-bit max/min, two chains) and over the
//           group's P lanes, then computes the group's parameters (the streaming kernel's
//           group_range / params_from_range: the same verified arithmetic) into LDS;
//   pass 2  lane = 8 consecutive elements (one qweight word at 4 bits): parameters from LDS
//           per half (L % 4 == 0) or per element, the field chain (bf16: packed f32 mul /
//           add), one coalesced word store.
// Tile boundaries fall on qweight and qzeros word boundaries (GPT * L and GPT are multiples
// of 8), so no word is shared between waves.  Replaces the one-wave-per-group generic
// kernel plus its int32 staging and pack passes (~10.5 B moved per element) for these
// shapes.
// ---------------------------------------------------------------------------------------
constexpr int kRgStageBytes = 8192;    // eligibility: 8 groups fit (any GPT the cost model picks)
constexpr int kRgStageMax = 16384;     // tuning override ceiling (rg_gpt)

template <typename F>
struct RgSlot {
    typedef typename std::conditional<F::kBytes == 2, uint16_t, uint32_t>::type T;
    static constexpr uint32_t kNan = F::kBytes == 2 ? 0xFFFFu : 0xFFFFFFFFu;   // field code of NaN
    __device__ static int sext(uint32_t v) { return F::kBytes == 2 ? (int)(int16_t)v : (int)v; }
    __device__ static float dec(uint32_t v) { return F::kBytes == 2 ? F::dec(v) : __uint_as_float(v); }
};

// packed field (q - qmin) of one element of a group with a positive finite scale, before
// the round + clamp (pack8_cvt / field_q)
template <typename F, int BITS, bool SYM, bool PLAIN>
__device__ __forceinline__ float field1_fast(float x, float r, float z, float s) {
    constexpr float HALF = (float)(1 << (BITS - 1));
    const float t = PLAIN ? F::quot_plain(x, r) : F::quot(x, s, r);
    float u;
    if (SYM && F::kWide) u = __builtin_rintf(t) + HALF;
    else if (SYM) u = t + HALF;
    else u = F::rn(t + F::as_fmt(z));
    return u;
}

// the field's value: clamp(rint(u), 0, 2^BITS - 1)
template <int BITS>
__device__ __forceinline__ float field_q(float u) {
    return __builtin_fminf(__builtin_fmaxf(__builtin_rintf(u), 0.0f), (float)((1 << BITS) - 1));
}

// the same for 8 bf16 elements, multiply and add as packed f32 pairs (v_pk_mul_f32 /
// v_pk_add_f32: each half is the IEEE f32 op, rounded to bf16 after it as above)
template <int BITS, bool SYM>
__device__ __forceinline__ void field8_bf16(const float (&x)[8], const float (&r)[8], const float (&z)[8],
                                            float (&q)[8]) {
    constexpr float HALF = (float)(1 << (BITS - 1));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const f2 p = (f2){x[2 * i], x[2 * i + 1]} * (f2){r[2 * i], r[2 * i + 1]};
        const f2 t = {rn_bf16(p.x), rn_bf16(p.y)};
        f2 u;
        if (SYM) {
            u = t + (f2){HALF, HALF};                       // exact (as field1_fast)
        } else {
            const f2 a = t + (f2){z[2 * i], z[2 * i + 1]};
            u = (f2){rn_bf16(a.x), rn_bf16(a.y)};
        }
        q[2 * i] = u.x;
        q[2 * i + 1] = u.y;
    }
}

// raw-bits min/max over each aligned block of 2^lgP lanes (a group's lanes in pass 1):
// DPP quad / mirror steps and the row-pair swaps (wave-uniform lgP), every lane ends with
// its block's result
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ void rg_step(int& smax, uint32_t& umax, uint32_t& umin) {
    smax = max(smax, (int)dpp_mov<CTRL>((uint32_t)smax));
    umax = max(umax, dpp_mov<CTRL>(umax));
    umin = min(umin, dpp_mov<CTRL>(umin));
}
__device__ __forceinline__ void rg_reduce(int& smax, uint32_t& umax, uint32_t& umin, int lgP) {
    if (lgP >= 1) rg_step<0xB1>(smax, umax, umin);     // quad_perm [1,0,3,2]
    if (lgP >= 2) rg_step<0x4E>(smax, umax, umin);     // quad_perm [2,3,0,1]
    if (lgP >= 3) rg_step<0x141>(smax, umax, umin);    // row_half_mirror
    if (lgP >= 4) rg_step<0x140>(smax, umax, umin);    // row_mirror
    if (lgP >= 5) {                                    // rows 2k <-> 2k+1
        const auto a = __builtin_amdgcn_permlane16_swap((unsigned)smax, (unsigned)smax, false, false);
        const auto b = __builtin_amdgcn_permlane16_swap(umax, umax, false, false);
        const auto c = __builtin_amdgcn_permlane16_swap(umin, umin, false, false);
        smax = max((int)a[0], (int)a[1]);
        umax = max((uint32_t)b[0], (uint32_t)b[1]);
        umin = min((uint32_t)c[0], (uint32_t)c[1]);
    }
    if (lgP >= 6) {                                    // halves
        const auto a = __builtin_amdgcn_permlane32_swap((unsigned)smax, (unsigned)smax, false, false);
        const auto b = __builtin_amdgcn_permlane32_swap(umax, umax, false, false);
        const auto c = __builtin_amdgcn_permlane32_swap(umin, umin, false, false);
        smax = max((int)a[0], (int)a[1]);
        umax = max((uint32_t)b[0], (uint32_t)b[1]);
        umin = min((uint32_t)c[0], (uint32_t)c[1]);
    }
}

#ifndef AWQ_RG_UNROLL
#define AWQ_RG_UNROLL 8
#endif

// raw-bits (signed max, unsigned max, unsigned min) of the 16-bit stage slots [s_lo, s_hi),
// s_hi > s_lo, from the identities: packed 16-bit max/min over whole dwords (two chains); an
// edge dword holding one foreign element gets a copy of its own element there
__device__ __forceinline__ void rg_range16(const uint32_t* st32, int s_lo, int s_hi, int& smax, uint32_t& umax,
                                           uint32_t& umin) {
    const int d_lo = s_lo >> 1, d_hi = (s_hi + 1) >> 1;
    s2 sm = {(short)-32768, (short)-32768}, sm_b = sm;
    us2 um = {0, 0}, um_b = um;
    us2 un = {(unsigned short)0xFFFF, (unsigned short)0xFFFF}, un_b = un;
    auto acc = [&](uint32_t v) {
        sm = __builtin_elementwise_max(sm, as_s2(v));
        um = __builtin_elementwise_max(um, as_us2(v));
        un = __builtin_elementwise_min(un, as_us2(v));
    };
    auto acc_b = [&](uint32_t v) {
        sm_b = __builtin_elementwise_max(sm_b, as_s2(v));
        um_b = __builtin_elementwise_max(um_b, as_us2(v));
        un_b = __builtin_elementwise_min(un_b, as_us2(v));
    };
    uint32_t first = st32[d_lo];
    if (s_lo & 1) first = __builtin_amdgcn_perm(first, first, 0x03020302u);   // low half := high
    if (d_hi - d_lo == 1 && (s_hi & 1)) first = __builtin_amdgcn_perm(first, first, 0x01000100u);
    acc(first);
    if (d_hi - d_lo > 1) {
        int d = d_lo + 1;
        for (; d + 4 <= d_hi - 1; d += 4) {
            const uint32_t v0 = st32[d], v1 = st32[d + 1], v2 = st32[d + 2], v3 = st32[d + 3];
            acc(v0);
            acc_b(v1);
            acc(v2);
            acc_b(v3);
        }
        if (d + 2 <= d_hi - 1) {
            const uint32_t v0 = st32[d], v1 = st32[d + 1];
            acc(v0);
            acc_b(v1);
            d += 2;
        }
        if (d < d_hi - 1) acc_b(st32[d]);
        uint32_t last = st32[d_hi - 1];
        if (s_hi & 1) last = __builtin_amdgcn_perm(last, last, 0x01000100u);        // high half := low
        acc(last);
    }
    sm = __builtin_elementwise_max(sm, sm_b);
    um = __builtin_elementwise_max(um, um_b);
    un = __builtin_elementwise_min(un, un_b);
    smax = max((int)sm.x, (int)sm.y);
    umax = (uint32_t)max((int)um.x, (int)um.y);
    umin = (uint32_t)min((int)un.x, (int)un.y);
}

// LDS: the segment's stage (dynamic, sized by the launch to the tile: 1.6-8 KiB) + 1.3 KiB
template <typename F, int BITS, bool SYM, int SPLIT, bool P1C>
__global__ __launch_bounds__(128) void awq_rowgroup_kernel(const void* __restrict__ w, int64_t rows, int64_t K,
                                                             int64_t L, int lgP, int GPT, uint32_t tiles_per_row,
                                                             int64_t G, int C, float invL,
                                                             int32_t* __restrict__ qweight, int32_t* __restrict__ qzeros,
                                                             uint16_t* __restrict__ scales,
                                                             int32_t* __restrict__ tensor_q, int32_t* __restrict__ zeros,
                                                             uint32_t nan_code) {
    typedef RgSlot<F> SL;
    typedef typename SL::T S;
    constexpr int QMIN = SYM ? -(1 << (BITS - 1)) : 0;
    constexpr uint32_t MASK = (1u << BITS) - 1u;
    constexpr int PER = 32 / BITS;             // elements (and groups) per packed word
    constexpr uint32_t NANF = (uint32_t)(0u - (uint32_t)QMIN) & MASK;   // field of INT32_MIN - qmin
    extern __shared__ __attribute__((aligned(16))) unsigned char rg_lds[];
    S* stage = (S*)rg_lds;                              // rg_stage_bytes(): the segment + its alignment skew
    __shared__ uint32_t zst[64];
    __shared__ float4 prm[64];                          // per group: r, z, s, special
    __shared__ int not_plain;                           // a group of the tile needs the full quotient
    __shared__ int acc_smax[P1C ? 64 : 1];              // P1C: per-group raw-bits reductions
    __shared__ uint32_t acc_umax[P1C ? 64 : 1], acc_umin[P1C ? 64 : 1];
    // one tile per workgroup of 1 or 2 waves (host-chosen: two waves share a large tile's LDS
    // stage, so a whole-row tile keeps 8 waves per SIMD resident)
    const int lane = threadIdx.x, NT = blockDim.x;
    // (host-side G, C, log2 P and a 32-bit tile split: 64-bit divisions per wave on the
    //  CU's shared scalar unit were a visible part of the per-tile cost)
    const uint32_t tile = blockIdx.x;   // (an XCD-contiguous tile order measured no different: r2z3)
    const uint32_t r32 = tile / tiles_per_row;
    const int64_t r = r32;
    const int64_t g0 = (int64_t)(tile - r32 * tiles_per_row) * GPT;
    const int ng = (int)min((int64_t)GPT, G - g0);
    if (ng < GPT) {   // the row's last, partial tile: more lanes per group (wave-uniform)
        lgP = min(6, 31 - __builtin_clz((unsigned)NT / (unsigned)ng));
        C = (int)((L + (1 << lgP) - 1) >> lgP);
    }
    const int P = 1 << lgP;
    const int64_t kb = g0 * L, ke = min((g0 + ng) * L, K);     // the row segment [kb, ke)
    const int n_el = (int)(ke - kb);
    // ---- stage the segment's bytes (from a 16-B aligned start) in LDS ----
    const uint64_t byte0 = (uint64_t)(r * K + kb) * F::kBytes;
    const uint64_t a0 = byte0 & ~(uint64_t)15;
    const int skew = (int)(byte0 - a0) / F::kBytes;               // slot of element kb
    const uint64_t total = (uint64_t)rows * (uint64_t)K * F::kBytes;
    const int nbytes = (int)(byte0 - a0) + n_el * F::kBytes;
    const int nch = (nbytes + 15) >> 4;
    const uint32_t lim = (uint32_t)min(total - a0, (uint64_t)nch * 16);
    const __amdgpu_buffer_rsrc_t rw = rsrc((const char*)w + a0, lim);
    if (__builtin_expect(16u * (uint32_t)nch <= lim, 1)) {
        // every 16-B load of the segment in flight before the first LDS store (a load ->
        // store loop waits out one memory round trip per load).  All 8 loads are issued
        // unconditionally: offsets past the segment fall outside the buffer range (lim) and
        // read zeros without a memory access, and no register needs a value on a skipped
        // path (conditional loads cost 28 v_mov per wave of phi copies); lanes past the end
        // store nothing
        for (int c0 = 0; c0 < nch; c0 += 8 * NT) {
            u4 v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k)
                v[k] = __builtin_amdgcn_raw_buffer_load_b128(rw, (uint32_t)(16 * (c0 + NT * k + lane)), 0, AWQ_LOAD_AUX);
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (c0 + NT * k + lane < nch) *(u4*)((char*)stage + 16 * (c0 + NT * k + lane)) = v[k];
        }
    } else
#pragma unroll 4
    for (int c = lane; c < nch; c += NT) {
        if (__builtin_expect(16u * c + 16u <= lim, 1)) {
            *(u4*)((char*)stage + 16 * c) = __builtin_amdgcn_raw_buffer_load_b128(rw, (uint32_t)(16 * c), 0, AWQ_LOAD_AUX);
        } else {   // the tensor's last bytes: a 16-B load straddling the range end would read as all zeros
            for (int h = 0; h < 8; ++h)
                ((uint16_t*)stage)[8 * c + h] = __builtin_amdgcn_raw_buffer_load_b16(rw, (uint32_t)(16 * c + 2 * h), 0, 0);
        }
    }
    if (lane == 0) not_plain = 0;
    if constexpr (P1C) {
        // identities; the row's zero-padded last group starts from 0 (awq.py:337-339: the
        // zeros join its min/max)
        if (lane < ng) {
            const bool pad = lane == ng - 1 && n_el - lane * (int)L < (int)L;
            acc_smax[lane] = pad ? 0 : INT_MIN;
            acc_umax[lane] = 0u;
            acc_umin[lane] = pad ? 0u : F::kOnes;
        }
    }
    __syncthreads();
    if constexpr (P1C) {
        // ---- pass 1, lanes split evenly over the tile's groups: Q = NT / ng lanes per group
        //      (any count — not only a power of two; 3 for 41 groups of a 128-lane tile where
        //      the by-groups pass keeps 2), each lane reduces one even-length run of its group
        //      and merges it into the group's LDS slots (ds_max / ds_min) ----
        const int Q = NT / ng;                            // >= 1: ng <= 64 <= NT
        const int grp = (int)((float)lane * __builtin_amdgcn_rcpf((float)Q) + 1e-3f);   // lane / Q (lane < 128)
        const int jq = lane - grp * Q;
        if (grp < ng) {
            const int glen = min((int)L, n_el - grp * (int)L);
            const int cq = ((glen + Q - 1) / Q + 1) & ~1;   // even: runs start on dword pairs
            const int cb = min(jq * cq, glen), ce = min(cb + cq, glen);
            if (ce > cb) {
                const int base = skew + grp * (int)L;
                int smx;
                uint32_t umx, umn;
                if constexpr (F::kBytes == 2) {
                    rg_range16((const uint32_t*)stage, base + cb, base + ce, smx, umx, umn);
                } else {
                    smx = INT_MIN;
                    umx = 0u;
                    umn = F::kOnes;
                    int i1 = cb;
                    for (; i1 + AWQ_RG_UNROLL <= ce; i1 += AWQ_RG_UNROLL) {
                        uint32_t v[AWQ_RG_UNROLL];
#pragma unroll
                        for (int u = 0; u < AWQ_RG_UNROLL; ++u) v[u] = stage[base + i1 + u];
#pragma unroll
                        for (int u = 0; u < AWQ_RG_UNROLL; ++u) {
                            smx = max(smx, SL::sext(v[u]));
                            umx = max(umx, v[u]);
                            umn = min(umn, v[u]);
                        }
                    }
                    for (; i1 < ce; ++i1) {
                        const uint32_t v = stage[base + i1];
                        smx = max(smx, SL::sext(v));
                        umx = max(umx, v);
                        umn = min(umn, v);
                    }
                }
                atomicMax(&acc_smax[grp], smx);
                atomicMax(&acc_umax[grp], umx);
                atomicMin(&acc_umin[grp], umn);
            }
        }
        __syncthreads();
        // ---- the tile's group parameters: one lane per group (wave 0: ng <= 64) ----
        if (lane < ng) {
            float gmn, gmx;
            bool gnan;
            group_range<F, SYM>(acc_smax[lane], acc_umax[lane], acc_umin[lane], gmn, gmx, gnan);
            const GroupParams p = params_from_range<F, BITS, SYM>(gmn, gmx);
            const bool special = !F::fast(p.r);
            if (F::kHasPlain && !F::plain_ok(p.s)) not_plain = 1;
            const int64_t gi = r * G + g0 + lane;
            if (scales) scales[gi] = f16_bits(p.s, gnan, nan_code);
            if (zeros) zeros[gi] = __builtin_isnan(p.z) ? INT32_MIN : (int32_t)p.z;
            zst[lane] = __builtin_isnan(p.z) ? NANF : ((uint32_t)((int)p.z - QMIN) & MASK);
            prm[lane] = (float4){p.r, p.z, p.s, special ? 1.0f : 0.0f};
        }
    } else {
    // ---- this lane's chunk of its group ----
    const int grp = lane >> lgP, j = lane & (P - 1);
    const bool active = grp < ng;
    const int glen = active ? min((int)L, n_el - grp * (int)L) : 0;   // elements in the row (tail: fewer)
    const int cb = min(j * C, glen), ce = min(cb + C, glen);
    const int base = skew + grp * (int)L;
    const bool padded = active && glen < L;                    // awq.py:337-339: zeros join the min/max
    int smax = padded ? 0 : INT_MIN;
    uint32_t umax = 0, umin = padded ? 0u : F::kOnes;
    if constexpr (F::kBytes == 2) {
        // raw 16-bit pairs with packed max/min (v_pk_*_i16/u16: two elements per instruction);
        // an edge dword holding one foreign element gets a copy of its own element there
        const int s_lo = base + cb, s_hi = base + ce;
        if (s_hi > s_lo) {
            const uint32_t* st32 = (const uint32_t*)stage;
            const int d_lo = s_lo >> 1, d_hi = (s_hi + 1) >> 1;
            s2 sm = {(short)(padded ? 0 : -32768), (short)(padded ? 0 : -32768)};
            us2 um = {0, 0};
            us2 un = {(unsigned short)(padded ? 0 : 0xFFFF), (unsigned short)(padded ? 0 : 0xFFFF)};
            s2 sm_b = sm;                                 // a second, independent set of chains
            us2 um_b = um, un_b = un;
            auto acc = [&](uint32_t v) {
                sm = __builtin_elementwise_max(sm, as_s2(v));
                um = __builtin_elementwise_max(um, as_us2(v));
                un = __builtin_elementwise_min(un, as_us2(v));
            };
            auto acc_b = [&](uint32_t v) {
                sm_b = __builtin_elementwise_max(sm_b, as_s2(v));
                um_b = __builtin_elementwise_max(um_b, as_us2(v));
                un_b = __builtin_elementwise_min(un_b, as_us2(v));
            };
            uint32_t first = st32[d_lo];
            if (s_lo & 1) first = __builtin_amdgcn_perm(first, first, 0x03020302u);   // low half := high
            if (d_hi - d_lo == 1 && (s_hi & 1)) first = __builtin_amdgcn_perm(first, first, 0x01000100u);
            acc(first);
            if (d_hi - d_lo > 1) {
                int d = d_lo + 1;
                for (; d + 4 <= d_hi - 1; d += 4) {
                    const uint32_t v0 = st32[d], v1 = st32[d + 1], v2 = st32[d + 2], v3 = st32[d + 3];
                    acc(v0);
                    acc_b(v1);
                    acc(v2);
                    acc_b(v3);
                }
                if (d + 2 <= d_hi - 1) {                  // <= 3 left: no loop
                    const uint32_t v0 = st32[d], v1 = st32[d + 1];
                    acc(v0);
                    acc_b(v1);
                    d += 2;
                }
                if (d < d_hi - 1) acc_b(st32[d]);
                uint32_t last = st32[d_hi - 1];
                if (s_hi & 1) last = __builtin_amdgcn_perm(last, last, 0x01000100u);        // high half := low
                acc(last);
            }
            sm = __builtin_elementwise_max(sm, sm_b);
            um = __builtin_elementwise_max(um, um_b);
            un = __builtin_elementwise_min(un, un_b);
            smax = max((int)sm.x, (int)sm.y);
            umax = (uint32_t)max((int)um.x, (int)um.y);
            umin = (uint32_t)min((int)un.x, (int)un.y);
        }
    } else {
        int i1 = cb;
        for (; i1 + AWQ_RG_UNROLL <= ce; i1 += AWQ_RG_UNROLL) {   // independent LDS reads in flight
            uint32_t v[AWQ_RG_UNROLL];
#pragma unroll
            for (int u = 0; u < AWQ_RG_UNROLL; ++u) v[u] = stage[base + i1 + u];
#pragma unroll
            for (int u = 0; u < AWQ_RG_UNROLL; ++u) {
                smax = max(smax, SL::sext(v[u]));
                umax = max(umax, v[u]);
                umin = min(umin, v[u]);
            }
        }
        for (; i1 < ce; ++i1) {
            const uint32_t v = stage[base + i1];
            smax = max(smax, SL::sext(v));
            umax = max(umax, v);
            umin = min(umin, v);
        }
    }
    rg_reduce(smax, umax, umin, lgP);                          // the group's P lanes (aligned)
    float gmn, gmx;
    bool gnan;
    group_range<F, SYM>(smax, umax, umin, gmn, gmx, gnan);
    const GroupParams p = params_from_range<F, BITS, SYM>(gmn, gmx);
    const bool special = !F::fast(p.r);
    // wave-uniform: every group of the tile admits the plain quotient (F::plain_ok)
    if (F::kHasPlain && active && j == 0 && !F::plain_ok(p.s)) not_plain = 1;
    if (active && j == 0) {
        const int64_t gi = r * G + g0 + grp;
        if (scales) scales[gi] = f16_bits(p.s, gnan, nan_code);
        if (zeros) zeros[gi] = __builtin_isnan(p.z) ? INT32_MIN : (int32_t)p.z;
        zst[grp] = __builtin_isnan(p.z) ? NANF : ((uint32_t)((int)p.z - QMIN) & MASK);
        prm[grp] = (float4){p.r, p.z, p.s, special ? 1.0f : 0.0f};
    }
    }   // (pass 1 by groups)
    __syncthreads();
    // uniform: every group of the tile admits the plain quotient (F::plain_ok)
    const bool plain = F::kHasPlain && not_plain == 0;
    // ---- pass 2: lane = 8 consecutive elements of the segment (one qweight word at 4 bits):
    //      its groups' parameters from LDS, quantize, pack, store (kb is a word boundary) ----
    const int nck = (n_el + 7) >> 3;
    const int L32 = (int)L;                               // invL = RN(1 / L): exact group index e * invL
                                                          // for e < 2^13, L <= 512 (host-computed)
    const int64_t wpr = (K + PER - 1) / PER;
    int32_t* qdst = qweight ? qweight + r * wpr + kb / PER : nullptr;
    float efA = 8.0f * (float)lane + 0.5f;                // e0c + 0.5 as an exact float induction
    const float efStep = 8.0f * (float)NT;
    for (int c = lane; c < nck; c += NT, efA += efStep) {
        const int e0c = 8 * c;
        const bool tail = e0c + 8 > n_el;                 // the row's last, partial chunk
        float x[8];
        if (skew == 0) {                                  // 16-B aligned chunk (K % 8 == 0 rows)
            const u4 v0 = *(const u4*)(stage + e0c);      // (past n_el: the stage's slack)
            if constexpr (F::kBytes == 2) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t wd = v0[i];
                    x[2 * i] = F::lo(wd);
                    x[2 * i + 1] = F::hi(wd);
                }
            } else {
                const u4 v1 = *(const u4*)(stage + e0c + 4);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    x[i] = __uint_as_float(v0[i]);
                    x[4 + i] = __uint_as_float(v1[i]);
                }
            }
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) x[i] = SL::dec(stage[skew + min(e0c + i, n_el - 1)]);
        }
        // parameters per element.  SPLIT 8 (L % 8 == 0): the chunk lies in one group; SPLIT 4
        // (L % 4 == 0): each half does (no per-element selects); SPLIT 1: at most two groups
        // meet in the chunk when L >= 8, one lookup per element below that
        float rr[8], zz[8], ss[8];
        bool spec;
        if constexpr (SPLIT == 8 || SPLIT == 4) {
            const int gA = (int)(efA * invL);             // < ng: e0c < n_el
            const float4 pA = prm[gA];
            float4 pB = pA;
            if constexpr (SPLIT == 4) pB = prm[min((int)((efA + 4.0f) * invL), ng - 1)];
            spec = pA.w != 0.0f || pB.w != 0.0f;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                rr[i] = i < 4 ? pA.x : pB.x;
                zz[i] = i < 4 ? pA.y : pB.y;
                ss[i] = i < 4 ? pA.z : pB.z;
            }
        } else if (L32 >= 8) {
            const int gA = (int)(((float)e0c + 0.5f) * invL);
            const int bnd = (gA + 1) * L32 - e0c;         // first element of the next group
            const float4 pA = prm[gA], pB = prm[min(gA + 1, ng - 1)];
            spec = pA.w != 0.0f || (bnd < 8 && pB.w != 0.0f);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const bool a = i < bnd;
                rr[i] = a ? pA.x : pB.x;
                zz[i] = a ? pA.y : pB.y;
                ss[i] = a ? pA.z : pB.z;
            }
        } else {
            spec = false;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int gi = min((int)(((float)(e0c + i) + 0.5f) * invL), ng - 1);
                const float4 pi = prm[gi];
                spec |= pi.w != 0.0f;
                rr[i] = pi.x;
                zz[i] = pi.y;
                ss[i] = pi.z;
            }
        }
        int32_t qv[8];                                    // q (reference value), INT32_MIN for NaN
        uint32_t word0 = 0, word1 = 0;
        if (__builtin_expect(!spec, 1)) {
            float q[8];
            if constexpr (std::is_same<F, FmtBF16>::value) {
                field8_bf16<BITS, SYM>(x, rr, zz, q);
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    q[i] = plain ? field1_fast<F, BITS, SYM, true>(x[i], rr[i], zz[i], ss[i])
                                 : field1_fast<F, BITS, SYM, false>(x[i], rr[i], zz[i], ss[i]);
            }
            if (__builtin_expect(tail, 0)) {
                const int nv = n_el - e0c;
#pragma unroll
                for (int i = 1; i < 8; ++i)
                    if (i >= nv) q[i] = 0.0f;             // past the row end: zero fields
            }
            if (tensor_q) {
#pragma unroll
                for (int i = 0; i < 8; ++i) qv[i] = (int32_t)field_q<BITS>(q[i]) + QMIN;
            }
            pack8_cvt<BITS>(q, word0, word1);
        } else {                                          // a group with scale 0 / inf / NaN: IEEE division
            constexpr int QMAX = SYM ? (1 << (BITS - 1)) - 1 : (1 << BITS) - 1;
            const int nv = n_el - e0c;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const float t = F::rn(opaque(x[i]) / ss[i]);
                const float u = SYM ? t : F::rn(t + zz[i]);
                const float rq = __builtin_rintf(u);
                int32_t qi = __builtin_isnan(rq) ? INT32_MIN
                                                 : (int32_t)__builtin_fminf(__builtin_fmaxf(rq, (float)QMIN), (float)QMAX);
                uint32_t f = ((uint32_t)qi - (uint32_t)QMIN) & MASK;
                if (i >= nv) { f = 0; qi = QMIN; }
                qv[i] = qi;
                if (BITS == 4) word0 |= f << (4 * i);
                else if (i < 4) word0 |= f << (8 * i);
                else word1 |= f << (8 * (i - 4));
            }
        }
        if (qdst) {
            if (BITS == 4) {
                qdst[c] = (int32_t)word0;
            } else {
                qdst[2 * c] = (int32_t)word0;
                if (!tail || e0c + 4 < n_el) qdst[2 * c + 1] = (int32_t)word1;
            }
        }
        if (tensor_q) {
            int32_t* tq = tensor_q + r * K + kb + e0c;
            if (__builtin_expect(!tail, 1)) {
#pragma unroll
                for (int i = 0; i < 8; ++i) tq[i] = qv[i];
            } else {
                const int nv = n_el - e0c;
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    if (i < nv) tq[i] = qv[i];
            }
        }
    }
    if (qzeros) {                                 // g0 is a word boundary: GPT % PER == 0
        const int64_t zpr = (G + PER - 1) / PER;
        const int nwz = (ng + PER - 1) / PER;
        if (lane < nwz) {
            uint32_t word = 0;
            for (int i = 0; i < PER && lane * PER + i < ng; ++i) word |= zst[lane * PER + i] << (BITS * i);
            qzeros[r * zpr + g0 / PER + lane] = (int32_t)word;
        }
    }
}

// Index of the tensor owning tile t, searching descs[base..n) (tile_begin ascending,
// descs[base].tile_begin <= t).  64 lanes probe 64 evenly spaced descriptors per round
// and a ballot narrows the range: one dependent load per round, 1 round for <= 64
// candidates, 2 for <= 4096 — instead of a chain of scalar loads through every tiny
// tensor (a model has ~100 1-tile bias tensors next to each other).
[[maybe_unused]] __device__ __forceinline__ int find_tensor(const awq_tensor_desc* __restrict__ descs, int n, int base,
                                           int64_t t) {
    const int lane = threadIdx.x & 63;
    int span = n - base;
    while (span > 1) {
        const int stride = (span + 63) >> 6;
        const int idx = base + lane * stride;
        const bool ok = (idx < base + span) && descs[min(idx, n - 1)].tile_begin <= t;
        const int cnt = __builtin_popcountll(__ballot(ok));   // ok lanes form a prefix
        base += (cnt - 1) * stride;
        span = min(stride, n - base);
    }
    return __builtin_amdgcn_readfirstlane(base);
}

#ifdef AWQ_TRACE
__device__ uint64_t* g_trace = nullptr;
#endif

// One wave per tile.  The grid normally covers every tile once (launch_fast); a smaller
// grid (awq_hip_tuning.h max_blocks, tests) makes each wave walk tiles t, t + nwaves, ... with a
// tensor cursor.
template <typename F, int BITS, bool SYM, bool SEARCH, int GS, bool PAD>
__global__ __launch_bounds__(64 * kWavesPerBlock, SEARCH ? 4 : (F::kWide ? AWQ_MIN_WAVES_WIDE : AWQ_MIN_WAVES))
void awq_fast_kernel(
    // the scalars every wave needs first lead the argument block (they fit the kernarg
    // preload window of a -mllvm -amdgpu-kernarg-preload-count build); the 80-B single-
    // tensor descriptor goes last
    const int32_t* __restrict__ block_tensor, const awq_tensor_desc* __restrict__ descs, int64_t total_tiles,
    int n, int n_grid, int n_cand, uint32_t nan_code, awq_tensor_desc single) {
    __shared__ uint32_t zwords[kWavesPerBlock][kTileElems / GS];
#if AWQ_WIDE_STORE
    __shared__ __attribute__((aligned(16))) uint32_t qstage_all[kWavesPerBlock][BITS == 4 ? 256 : 512];
#endif
    // wave index made provably uniform so tile/tensor bookkeeping and the buffer
    // descriptors live in SGPRs (no waterfall loops around the descriptors)
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * kWavesPerBlock;
    int64_t blk = blockIdx.x;
    if (AWQ_XCD_RUN > 0 && nwaves >= total_tiles) blk = xcd_run_block(blk, gridDim.x);   // one-shot grid only
    const int64_t wave = blk * kWavesPerBlock + wid;
    if (wave >= total_tiles) return;
    uint32_t* zw = zwords[wid];
#if AWQ_WIDE_STORE
    uint32_t* qs = qstage_all[wid];
#else
    uint32_t* qs = nullptr;
#endif
#ifdef AWQ_TRACE
    // timing-only build: per wave (start, first tile's loads issued, landed, end) in
    // s_memrealtime ticks (100 MHz, chip-wide clock) -> scripts/trace_waves.py
    const uint64_t tr0 = __builtin_amdgcn_s_memrealtime();
    uint64_t tr1 = 0, tr2 = 0;
#endif
    int cur = 0;
    awq_tensor_desc d = single;
    // the current tensor's input, first tile and shape: what the loads need (from the
    // table entry on a wave's first tile, else from the descriptor)
    const void* src_w = single.w;
    int64_t src_tb = single.tile_begin, src_rows = single.rows, src_K = single.K;
    bool need_d = false;   // d not loaded yet (fast table path): fetched after the loads went out
    if (descs != nullptr) {
        bool fast = false;
        if (block_tensor != nullptr) {
            // host-planned entry of the wave's tile group (awq_plan_block_tensor): ONE 64-B
            // scalar load gives the tensor's input and shape; entries whose tiles span
            // tensors (small tensors) step through the descriptors
            const TableEntry* te = (const TableEntry*)block_tensor + table_index(wave);
            const int32_t e = __builtin_amdgcn_readfirstlane(te->tensor);
            cur = e & 0x7FFFFFFF;
            if (e >= 0) {
                fast = true;
                src_w = te->w;
                src_tb = te->tile_begin;
                src_rows = te->rows;
                src_K = te->K;
                need_d = true;
            } else {
                while (cur + 1 < n && descs[cur + 1].tile_begin <= wave) ++cur;
            }
        } else {
            cur = find_tensor(descs, n, 0, wave);
        }
        if (!fast) {
            d = descs[cur];
            src_w = d.w;
            src_tb = d.tile_begin;
            src_rows = d.rows;
            src_K = d.K;
        }
    }
    for (int64_t t = wave; t < total_tiles; t += nwaves) {
        if (descs != nullptr && t != wave && cur + 1 < n && descs[cur + 1].tile_begin <= t) {
            cur = find_tensor(descs, n, cur + 1, t);
            d = descs[cur];
            need_d = false;
            src_w = d.w;
            src_tb = d.tile_begin;
            src_rows = d.rows;
            src_K = d.K;
        }
        // the input range first (no division for byte tiles): the loads go out before the
        // rest of the tile context (row / group divisions) is computed
        const uint32_t tile = (uint32_t)(t - src_tb);
        uint64_t el_off;
        uint32_t valid;
        tile_src<BITS, GS, PAD>(src_rows, src_K, tile, el_off, valid);
        Chunk<F::NW> va[4];
        load_tile<F, GS>((const char*)src_w + el_off * F::kBytes, valid, va);
        if (need_d) {   // the descriptor (outputs) while the loads are in flight
            d = descs[cur];
            need_d = false;
        }
#ifdef AWQ_TRACE
        if (tr1 == 0) {
            tr1 = __builtin_amdgcn_s_memrealtime();
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            tr2 = __builtin_amdgcn_s_memrealtime();
        }
#endif
        compute_tile<F, BITS, SYM, SEARCH, GS>(make_ctx<BITS, GS, PAD>(d, tile), va, zw, qs, n_grid, n_cand, nan_code);
    }
#ifdef AWQ_TRACE
    if (g_trace != nullptr && (threadIdx.x & 63) == 0) {
        g_trace[wave * 4 + 0] = tr0;
        g_trace[wave * 4 + 1] = tr1;
        g_trace[wave * 4 + 2] = tr2;
        g_trace[wave * 4 + 3] = __builtin_amdgcn_s_memrealtime();
    }
#endif
}

// Exhaustive self-test of recip_bf16 over every non-negative bf16 bit pattern
// s >= RN_bf16(1e-10) (incl. inf / NaN): counts results that differ bitwise from the
// IEEE division.
__global__ void awq_selftest_recip_kernel(unsigned long long* mismatches) {
    const uint32_t h = blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= 0x8000u) return;
    const float s = __uint_as_float(h << 16);
    if (!(s >= __uint_as_float(0x2EDC0000u)) && !__builtin_isnan(s)) return;
    const float a = recip_bf16(s);
    const float b = 1.0f / s;
    if (__float_as_uint(a) != __float_as_uint(b) && !(__builtin_isnan(a) && __builtin_isnan(b)))
        atomicAdd(mismatches, 1ull);
}

}  // namespace

hipError_t launch_fast(const awq_tensor_desc* descs_dev, const int32_t* block_tensor,
                       const awq_tensor_desc* single, int n, int64_t total_tiles, int dtype, int bits,
                       int symmetric, int group_size, bool padded, hipStream_t stream, uint32_t nan_code, int n_grid,
                       int n_cand) {
    if (total_tiles <= 0) return hipSuccess;
    // one wave per tile (diagnostics, include/awq_hip_tuning.h: tiles_per_wave, max_blocks =
    // grid cap; either makes waves walk several tiles)
    int64_t tpw = 1, max_blocks = INT32_MAX;
    if (tuning().tiles_per_wave > 1) tpw = tuning().tiles_per_wave;
    if (tuning().max_blocks > 0) max_blocks = tuning().max_blocks;
    const int64_t per_block = kWavesPerBlock * tpw;
    int64_t blocks = (total_tiles + per_block - 1) / per_block;
    if (blocks > max_blocks) blocks = max_blocks;
    awq_tensor_desc one{};
    if (single) one = *single;
    // the table is indexed by the wave's first tile: valid for the one-tile-per-wave grid only
    const int32_t* bt = (tpw == 1 && blocks * per_block >= total_tiles) ? block_tensor : nullptr;
    const dim3 grid((unsigned)blocks), block(64 * kWavesPerBlock);
#define AWQ_LAUNCH_GS(Fm, B, S, G)                                                                                  \
    do {                                                                                                            \
        if (n_cand > 1 && padded)                                                                                   \
            hipLaunchKernelGGL((awq_fast_kernel<Fm, B, S, true, G, true>), grid, block, 0, stream, bt, descs_dev,   \
                               total_tiles, n, n_grid, n_cand, nan_code, one);                                                \
        else if (n_cand > 1)                                                                                        \
            hipLaunchKernelGGL((awq_fast_kernel<Fm, B, S, true, G, false>), grid, block, 0, stream, bt, descs_dev,  \
                               total_tiles, n, n_grid, n_cand, nan_code, one);                                                \
        else if (padded)                                                                                            \
            hipLaunchKernelGGL((awq_fast_kernel<Fm, B, S, false, G, true>), grid, block, 0, stream, bt, descs_dev,  \
                               total_tiles, n, 1, 0, nan_code, one);                                                          \
        else                                                                                                        \
            hipLaunchKernelGGL((awq_fast_kernel<Fm, B, S, false, G, false>), grid, block, 0, stream, bt, descs_dev, \
                               total_tiles, n, 1, 0, nan_code, one);                                                          \
    } while (0)
#define AWQ_LAUNCH(Fm, B, S)                                   \
    switch (group_size) {                                      \
    case 32: AWQ_LAUNCH_GS(Fm, B, S, 32); break;               \
    case 64: AWQ_LAUNCH_GS(Fm, B, S, 64); break;               \
    case 256: AWQ_LAUNCH_GS(Fm, B, S, 256); break;             \
    default: AWQ_LAUNCH_GS(Fm, B, S, 128); break;              \
    }
#define AWQ_LAUNCH_FMT(Fm)                          \
    switch ((bits == 8 ? 2 : 0) + (symmetric ? 1 : 0)) { \
    case 0: AWQ_LAUNCH(Fm, 4, false); break;        \
    case 1: AWQ_LAUNCH(Fm, 4, true); break;         \
    case 2: AWQ_LAUNCH(Fm, 8, false); break;        \
    default: AWQ_LAUNCH(Fm, 8, true); break;        \
    }
    if (!fast_group_size(group_size)) return hipErrorInvalidValue;
    if (dtype == AWQ_DTYPE_F16) {
        AWQ_LAUNCH_FMT(FmtF16)
    } else if (dtype == AWQ_DTYPE_F32) {
        AWQ_LAUNCH_FMT(FmtF32)
    } else {
        AWQ_LAUNCH_FMT(FmtBF16)
    }
#undef AWQ_LAUNCH_FMT
#undef AWQ_LAUNCH
#undef AWQ_LAUNCH_GS
    return hipPeekAtLastError();
}

// Row-segment tiles of awq_rowgroup_kernel.  Whole-row tiles shared by two waves when a
// 16-bit row of >= 2560 elements has <= 64 groups and fits a 16 KiB stage (r2ae / r2af: a
// whole-row tile runs 1 059 VALU per row against 1 551 for 16-group one-wave tiles, and two
// waves per LDS stage keep the SIMDs occupied; r2ag: +8..44 % at K = 3000 / 4096, e.g. bf16
// gs 100 47.6 -> 42.5 us; -10..15 % at K = 2048, hence the threshold).  Otherwise one wave per tile and GPT (8..64, a power of two) from a
// per-row cost fitted to measurements (profiles/round2/r2_rowgroup/r2r_*: 14336 x 4096,
// group sizes 48 / 100, GPT 8..32): tiles x (fixed wave cost 8 + 0.6 per element of a
// lane's pass-1 chunk C = L / (64 / GPT) + 2.3 per 512-element pass-2 sweep).  gpt = 0 if
// the shape does not fit the LDS stage.  rg_gpt / rg_waves override (awq_hip_tuning.h).
struct RgPlan {
    int gpt, waves;
};
RgPlan rowgroup_plan(int dtype, int64_t K, int64_t L) {
    RgPlan pl = {0, 1};
    if (dtype != AWQ_DTYPE_BF16 && dtype != AWQ_DTYPE_F16 && dtype != AWQ_DTYPE_F32) return pl;
    const int64_t es = dtype == AWQ_DTYPE_F32 ? 4 : 2;
    // (L = 1: a one-element group's NaN scale keeps the element's own NaN bits — generic kernel)
    if (L < 2 || K <= 0 || 8 * L * es > kRgStageBytes) return pl;
    const bool ew = tuning().rg_waves == 1 || tuning().rg_waves == 2;
    if (ew) pl.waves = tuning().rg_waves;
    if (const int v = tuning().rg_gpt) {
        if (v >= 8 && v <= 64 && v % 8 == 0 && v * L * es <= kRgStageMax) {
            pl.gpt = v;
            return pl;
        }
    }
    const int64_t G = (K + L - 1) / L;
    const int64_t whole = (G + 7) / 8 * 8;
    if (!ew && es == 2 && K >= 2560 && whole <= 64 && whole * L * es <= kRgStageMax) {
        pl.gpt = (int)whole;
        pl.waves = 2;
        return pl;
    }
    double best_cost = 0.0;
    for (int gpt = 8; gpt <= 64; gpt *= 2) {
        if (gpt * L * es > kRgStageBytes) break;
        const int64_t tiles = (G + gpt - 1) / gpt;
        const int64_t C = (L + (64 / gpt) - 1) / (64 / gpt);
        const int64_t el = min((int64_t)gpt, G) * L;                  // elements of a full tile
        const double cost = (double)tiles * (8.0 + 0.6 * (double)C + 2.3 * (double)((el + 511) / 512));
        if (pl.gpt == 0 || cost < best_cost) { best_cost = cost; pl.gpt = gpt; }
    }
    return pl;
}
int rowgroup_gpt(int dtype, int64_t K, int64_t L) { return rowgroup_plan(dtype, K, L).gpt; }

hipError_t launch_rowgroup(const void* w, int dtype, int64_t rows, int64_t K, int64_t L, int bits, int symmetric,
                           int32_t* qweight, int32_t* qzeros, uint16_t* scales, int32_t* tensor_q, int32_t* zeros,
                           hipStream_t stream, uint32_t nan_code) {
    const RgPlan pl = rowgroup_plan(dtype, K, L);
    const int gpt = pl.gpt;
    if (gpt == 0 || rows <= 0) return hipErrorInvalidValue;
    const int64_t G = (K + L - 1) / L;
    const int64_t tpr = (G + gpt - 1) / gpt;
    const int nt = 64 * pl.waves;                                      // threads per tile
    const int lgP = min(6, 31 - __builtin_clz((unsigned)(nt / gpt)));  // P = lanes per group: a power of two
    const int P = 1 << lgP;
    const int C = (int)((L + P - 1) / P);
    const dim3 grid((unsigned)(rows * tpr)), block((unsigned)nt);
    // stage: the tile's elements rounded up to 16 B, + the up-to-16-B alignment skew and the
    // last 8-element vector read past the segment end
    const size_t lds = ((size_t)gpt * L * (dtype == AWQ_DTYPE_F32 ? 4 : 2) + 15) / 16 * 16 + 48;
    const bool p1c = tuning().rg_p1 == 2;   // pass 1 by groups (default) / evenly split runs (A/B)
#define AWQ_RG_SPLIT(Fm, B, S, SP)                                                                                 \
    do {                                                                                                           \
        if (p1c)                                                                                                   \
            hipLaunchKernelGGL((awq_rowgroup_kernel<Fm, B, S, SP, true>), grid, block, lds, stream, w, rows, K, L, \
                               lgP, gpt, (uint32_t)tpr, G, C, 1.0f / (float)L, qweight, qzeros, scales, tensor_q,  \
                               zeros, nan_code);                                                                   \
        else                                                                                                       \
            hipLaunchKernelGGL((awq_rowgroup_kernel<Fm, B, S, SP, false>), grid, block, lds, stream, w, rows, K,   \
                               L, lgP, gpt, (uint32_t)tpr, G, C, 1.0f / (float)L, qweight, qzeros, scales,         \
                               tensor_q, zeros, nan_code);                                                         \
    } while (0)
#define AWQ_RG(Fm, B, S)                                                                                           \
    if (L % 8 == 0) AWQ_RG_SPLIT(Fm, B, S, 8);                                                                      \
    else if (L % 4 == 0) AWQ_RG_SPLIT(Fm, B, S, 4);                                                                 \
    else AWQ_RG_SPLIT(Fm, B, S, 1)
#define AWQ_RG_FMT(Fm)                                                     \
    switch ((bits == 8 ? 2 : 0) + (symmetric ? 1 : 0)) {                  \
    case 0: AWQ_RG(Fm, 4, false); break;                                   \
    case 1: AWQ_RG(Fm, 4, true); break;                                    \
    case 2: AWQ_RG(Fm, 8, false); break;                                   \
    default: AWQ_RG(Fm, 8, true); break;                                   \
    }
    if (dtype == AWQ_DTYPE_F16) {
        AWQ_RG_FMT(FmtF16)
    } else if (dtype == AWQ_DTYPE_F32) {
        AWQ_RG_FMT(FmtF32)
    } else {
        AWQ_RG_FMT(FmtBF16)
    }
#undef AWQ_RG_FMT
#undef AWQ_RG
#undef AWQ_RG_SPLIT
    return hipPeekAtLastError();
}

#ifdef AWQ_TRACE
extern "C" int awq_debug_set_trace(void* buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &buf, sizeof(buf)) == hipSuccess ? 0 : 1;
}
#endif

// Measurement helper (bench.py's copy ceiling): a plain HBM copy with the quantizer's
// memory structure — one wave per 4 KiB, 4 x 16-B nt loads and stores per lane, the same
// one-wave-per-tile grid of 512-thread workgroups.  Read + write bytes = 2 x `bytes`.
__global__ __launch_bounds__(64 * kWavesPerBlock) void awq_stream_copy_kernel(const uint8_t* __restrict__ src,
                                                                             uint8_t* __restrict__ dst,
                                                                             int64_t bytes) {
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t base = ((int64_t)blockIdx.x * kWavesPerBlock + wid) * 4096;
    if (base >= bytes) return;
    const uint32_t n = (uint32_t)min((int64_t)4096, bytes - base);
    const __amdgpu_buffer_rsrc_t rs = rsrc(src + base, n), rd = rsrc(dst + base, n);
    u4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(j * 1024 + lane * 16), 0, 2);
#pragma unroll
    for (int j = 0; j < 4; ++j) __builtin_amdgcn_raw_buffer_store_b128(v[j], rd, (uint32_t)(j * 1024 + lane * 16), 0, 2);
}

hipError_t launch_stream_copy(const void* src, void* dst, int64_t bytes, hipStream_t stream) {
    if (bytes <= 0) return hipSuccess;
    const int64_t per_block = 4096LL * kWavesPerBlock;
    hipLaunchKernelGGL(awq_stream_copy_kernel, dim3((unsigned)((bytes + per_block - 1) / per_block)),
                       dim3(64 * kWavesPerBlock), 0, stream, (const uint8_t*)src, (uint8_t*)dst, bytes);
    return hipPeekAtLastError();
}

// Measurement helper (bench.py's read-dominant ceiling): the quantizer's memory structure
// and read:write ratio without its arithmetic — one wave per 4 KiB of input (4 x 16-B nt
// loads per lane), the four vectors xor-folded to one, ONE 16-B nt store per lane (1 KiB
// per wave).  Read 4 : write 1, against the packed quantizer's 4096 : 1064 per tile.
__global__ __launch_bounds__(64 * kWavesPerBlock) void awq_stream_ceiling_kernel(const uint8_t* __restrict__ src,
                                                                                uint8_t* __restrict__ dst,
                                                                                int64_t bytes) {
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t tile = (int64_t)blockIdx.x * kWavesPerBlock + wid;
    const int64_t base = tile * 4096;
    if (base >= bytes) return;
    const uint32_t n = (uint32_t)min((int64_t)4096, bytes - base);
    const __amdgpu_buffer_rsrc_t rs = rsrc(src + base, n), rd = rsrc(dst + tile * 1024, n / 4);
    u4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(j * 1024 + lane * 16), 0, 2);
    const u4 x = v[0] ^ v[1] ^ v[2] ^ v[3];
    __builtin_amdgcn_raw_buffer_store_b128(x, rd, (uint32_t)(lane * 16), 0, 2);
}

hipError_t launch_stream_ceiling(const void* src, void* dst, int64_t bytes, hipStream_t stream) {
    if (bytes <= 0) return hipSuccess;
    const int64_t per_block = 4096LL * kWavesPerBlock;
    hipLaunchKernelGGL(awq_stream_ceiling_kernel, dim3((unsigned)((bytes + per_block - 1) / per_block)),
                       dim3(64 * kWavesPerBlock), 0, stream, (const uint8_t*)src, (uint8_t*)dst, bytes);
    return hipPeekAtLastError();
}

hipError_t launch_selftest(int which, unsigned long long* out, hipStream_t stream) {
    if (which != 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(awq_selftest_recip_kernel, dim3(0x8000 / 256), dim3(256), 0, stream, out);
    return hipPeekAtLastError();
}

}  // namespace awq
