// awq_actsearch.hip — activation-aware per-input-channel scale search (scale_method="awq").
//
// No reference counterpart: the reference stores scale_method and never reads it
// (awq.py:66,111-112) and collects no activations (SURVEY.md §1, §8a "parity unpinned").
// This is the search AutoAWQ publishes (per input channel k, s_k = x_mean_k^r, optionally
// divided by w_mean_k^(1-r) ("duo scaling"), normalised, r = i / n_grid; quantize W·diag(s),
// undo s, keep the r with the smallest error), with its output-MSE loss
// ||X (Ŵ - W)^T||² replaced by the diagonal form Σ_k E[x_k²] Σ_n (Ŵ_nk - W_nk)² — exact
// for uncorrelated input channels, computable per element, so the whole search is one
// streaming pass over W (all candidates evaluated from registers) instead of n_grid GEMMs.
// Definition, canonical summation orders and ABI: include/awq_hip.h (awq_act_*); CPU
// restatement: oracle/awq_oracle.c (oracle_act_*).
//
// Every element-wise op follows the reference recipe for the weight dtype D (refmath:
// fp32 math, RNE to D after each op); the scale table is computed in fp64.
#include "awq_refmath.h"

namespace awq {
namespace {

using namespace refmath;

typedef float f2 __attribute__((ext_vector_type(2)));
typedef __bf16 b2 __attribute__((ext_vector_type(2)));

// ---- hardware-conversion arithmetic for bf16 / fp16 weights (the streaming kernel's
// verified identities, awq_fast.hip): same results as refmath, ~4x fewer VALU ----
__device__ __forceinline__ float opq(float a) {   // value barrier: no f16 narrowing / mixlo fusion
    asm volatile("" : "+v"(a));
    return a;
}
__device__ __forceinline__ float hw_rn_bf16(float a) {   // v_cvt_pk_bf16_f32: RNE, NaN stays NaN
    b2 h = __builtin_convertvector((f2){0.0f, a}, b2);
    return __builtin_bit_cast(float, h);
}
__device__ __forceinline__ float hw_rn_f16(float a) { return (float)(_Float16)opq(a); }   // v_cvt_f16_f32: RNE

// RN_f32(1/s) for a bf16-valued s: v_rcp_f32 + one Newton step, correctly rounded for every
// bf16 s < 2^126 (awq_selftest checks all of them against IEEE 1/s); IEEE division beyond
__device__ __forceinline__ float recip_bf16(float s) {
    if (__builtin_expect(!(s < 0x1p126f), 0)) return 1.0f / s;
    const float r0 = __builtin_amdgcn_rcpf(s);
    const float e = __builtin_fmaf(-s, r0, 1.0f);
    return __builtin_fmaf(r0, e, r0);
}

template <int DT> struct HwFmt;
template <> struct HwFmt<AWQ_DTYPE_BF16> {
    __device__ static float lo() { return __uint_as_float(0x2EDC0000u); }   // RN_bf16(1e-10)
    // RN(d / qr) for bf16 d, qr in {15, 255}: d * RN(1/qr) (the same exhaustive identity)
    __device__ static float scale(float d, float qr, float rq) {
        (void)qr;
        return hw_rn_bf16(d * rq);
    }
    __device__ static float recip(float s) { return recip_bf16(s); }
    // RN(x / s) for any s >= RN(1e-10) incl. inf / NaN (r = 0 / NaN carries them)
    __device__ static float quot_any(float x, float s, float r) {
        (void)s;
        return hw_rn_bf16(x * r);
    }
    __device__ static float rn(float a) { return hw_rn_bf16(a); }
    // RN(x / s) = RN_bf16(x * RN_f32(1/s)) for bf16 x and bf16 s >= RN_bf16(1e-10)
    // (exhaustive, oracle/verify_recip.c)
    __device__ static float quot(float x, float s, float r) {
        (void)s;
        return hw_rn_bf16(x * r);
    }
};
// AWQ_F16_PARAMS_FAST = 0: the fp16 group parameters by IEEE divisions (as csrc/awq_quant.h)
#ifndef AWQ_F16_PARAMS_FAST
#define AWQ_F16_PARAMS_FAST 1
#endif
// rcp + one Newton step: IEEE 1/s for every positive finite fp16 s (awq_selftest 2)
__device__ __forceinline__ float recip_f16(float s) {
    if (__builtin_expect(!(s > 0.0f && s < __builtin_inff()), 0)) return 1.0f / s;
    const float r0 = __builtin_amdgcn_rcpf(s);
    const float e = __builtin_fmaf(-s, r0, 1.0f);
    return __builtin_fmaf(r0, e, r0);
}
template <> struct HwFmt<AWQ_DTYPE_F16> {
    __device__ static float lo() { return 0.0f; }                           // RN_f16(1e-10) = 0
#if AWQ_F16_PARAMS_FAST
    // RN_f16(d / qr) == RN_f16(d * RN_f32(1/qr)), every non-negative fp16 d incl. inf
    // (oracle/verify_recip.c f16scale)
    __device__ static float scale(float d, float qr, float rq) {
        (void)qr;
        return hw_rn_f16(opq(hw_rn_f16(d)) * rq);
    }
    __device__ static float recip(float s) { return recip_f16(s); }
    // the Markstein quotient for a positive finite s (verify_recip f16m), IEEE otherwise
    __device__ static float quot_any(float x, float s, float r) {
        if (__builtin_expect(!(s > 0.0f && s < __builtin_inff()), 0)) return hw_rn_f16(opq(x) / s);
        return quot(x, s, r);
    }
#else
    __device__ static float scale(float d, float qr, float rq) {   // IEEE: d may be inf (Markstein would NaN)
        (void)rq;
        return hw_rn_f16(opq(d) / qr);
    }
    __device__ static float recip(float s) { return 1.0f / s; }
    __device__ static float quot_any(float x, float s, float r) {          // IEEE: s may be 0 / inf / NaN
        (void)r;
        return hw_rn_f16(opq(x) / s);
    }
#endif
    __device__ static float rn(float a) { return hw_rn_f16(a); }
    // Markstein-corrected quotient, exact for every fp16 x and positive finite fp16 s
    // (oracle/verify_recip.c f16m)
    __device__ static float quot(float x, float s, float r) {
        const float q0 = x * r;
        const float e = __builtin_fmaf(-s, q0, x);
        return hw_rn_f16(__builtin_fmaf(e, r, q0));
    }
};
// fp32 weights: every op is the fp32 op itself, x / s the IEEE division
template <> struct HwFmt<AWQ_DTYPE_F32> {
    __device__ static float lo() { return 1e-10f; }
    __device__ static float scale(float d, float qr, float rq) {
        (void)rq;
        return d / qr;
    }
    __device__ static float recip(float s) { return 1.0f / s; }
    __device__ static float quot_any(float x, float s, float r) {
        (void)r;
        return x / s;
    }
    __device__ static float rn(float a) { return a; }
    __device__ static float quot(float x, float s, float r) {
        (void)r;
        return x / s;
    }
};

// awq.py:196-213 with the hardware identities above (same results as refmath::group_params:
// qmin = 0 whenever the zero point is used, so RN(qmin - y) is exact, and rint of a value of
// the dtype is again a value of the dtype); also returns r = RN_f32(1 / s) for the element
// path.
template <int DT>
__device__ __forceinline__ void hw_group_params(float mn, float mx, int nan, int qmin, int qmax, int sym, float rq,
                                                float& s_out, float& z_out, float& r_out) {
    typedef HwFmt<DT> H;
    if (sym) {                                                // awq.py:196-199
        float amn = __builtin_fabsf(mn), amx = __builtin_fabsf(mx);
        if (nan) { amn = mn; amx = mx; }
        const float a = (amx > amn) ? amx : amn;
        mn = -a;
        mx = a;
    }
    float s = H::scale(H::rn(mx - mn), (float)(qmax - qmin), rq);   // awq.py:202
    if (!(s != s) && s < H::lo()) s = H::lo();                        // awq.py:205
    const float r = H::recip(s);
    float z = 0.0f;
    if (!sym)                                                 // awq.py:210-211
        z = clampq(__builtin_rintf((float)qmin - H::quot_any(mn, s, r)), (float)qmin, (float)qmax);
    s_out = s;
    z_out = z;
    r_out = r;
}

// Reductions over the lpg consecutive lanes of a group (lpg a power of two <= 64), every
// lane getting the result: DPP inside 16-lane rows (quad perms, half-row / row mirrors —
// after the earlier steps these pair exactly the lanes an xor butterfly pairs), permlane
// swaps across rows.  fmin/fmax skip NaN (NaN is tracked separately); the sum adds
// own + partner at every level like the xor butterfly (the canonical tree, include/awq_hip.h).
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
template <int CTRL>
__device__ __forceinline__ int dppi(int v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true);
}
// the two 16-lane rows (or 32-lane halves) of a pair, swapped: lane l sees {its pair's
// first half, its pair's second half} whichever half it is in, so combining p.x and p.y
// symmetrically (min, max, or, +) gives every lane f(own, partner) exactly
__device__ __forceinline__ void swap16(unsigned u, unsigned& a, unsigned& b) {
    const auto p = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    a = p[0];
    b = p[1];
}
__device__ __forceinline__ void swap32(unsigned u, unsigned& a, unsigned& b) {
    const auto p = __builtin_amdgcn_permlane32_swap(u, u, false, false);
    a = p[0];
    b = p[1];
}
__device__ __forceinline__ float fbits(unsigned u) { return __builtin_bit_cast(float, u); }
__device__ __forceinline__ unsigned ubits(float f) { return __builtin_bit_cast(unsigned, f); }

template <bool ROW32>
__device__ __forceinline__ void minmax_cross(float& mn, float& mx, int& nan) {
    unsigned a, b;
    if (ROW32) swap32(ubits(mn), a, b); else swap16(ubits(mn), a, b);
    mn = __builtin_amdgcn_fmed3f(fbits(a), fbits(b), -__builtin_inff());
    if (ROW32) swap32(ubits(mx), a, b); else swap16(ubits(mx), a, b);
    mx = __builtin_amdgcn_fmed3f(fbits(a), fbits(b), __builtin_inff());
    if (ROW32) swap32((unsigned)nan, a, b); else swap16((unsigned)nan, a, b);
    nan = (int)(a | b);
}

// min(a, b) / max(a, b) as v_med3 against -inf / +inf: no NaN-quieting of the DPP-moved
// operand (fminf / fmaxf need it in IEEE mode); NaN is tracked on the side, so no operand is
// NaN whenever the result is used
__device__ __forceinline__ float min2(float a, float b) { return __builtin_amdgcn_fmed3f(a, b, -__builtin_inff()); }
__device__ __forceinline__ float max2(float a, float b) { return __builtin_amdgcn_fmed3f(a, b, __builtin_inff()); }

__device__ __forceinline__ void grp_minmax(float& mn, float& mx, int& nan, int lpg) {
    if (lpg >= 2) { mn = min2(mn, dppf<0xB1>(mn)); mx = max2(mx, dppf<0xB1>(mx)); nan |= dppi<0xB1>(nan); }
    if (lpg >= 4) { mn = min2(mn, dppf<0x4E>(mn)); mx = max2(mx, dppf<0x4E>(mx)); nan |= dppi<0x4E>(nan); }
    if (lpg >= 8) { mn = min2(mn, dppf<0x141>(mn)); mx = max2(mx, dppf<0x141>(mx)); nan |= dppi<0x141>(nan); }
    if (lpg >= 16) { mn = min2(mn, dppf<0x140>(mn)); mx = max2(mx, dppf<0x140>(mx)); nan |= dppi<0x140>(nan); }
    if (lpg >= 32) minmax_cross<false>(mn, mx, nan);
    if (lpg >= 64) minmax_cross<true>(mn, mx, nan);
}

// v_min_f32 / v_max_f32 with the partner lane's operand through DPP, one instruction per step
// (the compiler turns min2 / max2 into v_min / v_max behind a canonicalising v_max x, x and a
// separate v_mov_dpp: three).  The s_nop covers the VALU-write -> DPP-read wait states (the
// operand may have been written by the instruction just before).  No NaN reaches these (the
// weights' NaN flag is tracked on the side), and the sign of a zero extreme cannot change the
// scale or zero point.
#define AWQ_DPP_MINMAX(NAME, OP, CTRL)                                                                   \
    __device__ __forceinline__ float NAME(float v) {                                                    \
        float r;                                                                                        \
        asm("s_nop 1\n\t" OP "_dpp %0, %1, %1 " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(r) : "v"(v)); \
        return r;                                                                                       \
    }
AWQ_DPP_MINMAX(min_xor1, "v_min_f32", "quad_perm:[1,0,3,2]")
AWQ_DPP_MINMAX(max_xor1, "v_max_f32", "quad_perm:[1,0,3,2]")
AWQ_DPP_MINMAX(min_xor2, "v_min_f32", "quad_perm:[2,3,0,1]")
AWQ_DPP_MINMAX(max_xor2, "v_max_f32", "quad_perm:[2,3,0,1]")
AWQ_DPP_MINMAX(min_hmir, "v_min_f32", "row_half_mirror")
AWQ_DPP_MINMAX(max_hmir, "v_max_f32", "row_half_mirror")
AWQ_DPP_MINMAX(min_mir, "v_min_f32", "row_mirror")
AWQ_DPP_MINMAX(max_mir, "v_max_f32", "row_mirror")
#undef AWQ_DPP_MINMAX
#ifndef AWQ_ACT_DPP_MINMAX
#define AWQ_ACT_DPP_MINMAX 1
#endif

// the group min / max alone (the weights' NaN flag is reduced once per item: grp_or)
__device__ __forceinline__ void grp_minmax_nn(float& mn, float& mx, int lpg) {
#if AWQ_ACT_DPP_MINMAX
    if (lpg >= 2) { mn = min_xor1(mn); mx = max_xor1(mx); }
    if (lpg >= 4) { mn = min_xor2(mn); mx = max_xor2(mx); }
    if (lpg >= 8) { mn = min_hmir(mn); mx = max_hmir(mx); }
    if (lpg >= 16) { mn = min_mir(mn); mx = max_mir(mx); }
    // the compiler's hazard tracking does not see into the asm: wait states before the cross-row
    // swaps below read its results
    if (lpg >= 32) asm volatile("s_nop 1" : "+v"(mn), "+v"(mx));
#else
    if (lpg >= 2) { mn = min2(mn, dppf<0xB1>(mn)); mx = max2(mx, dppf<0xB1>(mx)); }
    if (lpg >= 4) { mn = min2(mn, dppf<0x4E>(mn)); mx = max2(mx, dppf<0x4E>(mx)); }
    if (lpg >= 8) { mn = min2(mn, dppf<0x141>(mn)); mx = max2(mx, dppf<0x141>(mx)); }
    if (lpg >= 16) { mn = min2(mn, dppf<0x140>(mn)); mx = max2(mx, dppf<0x140>(mx)); }
#endif
    if (lpg >= 32) {
        int dummy = 0;
        minmax_cross<false>(mn, mx, dummy);
    }
    if (lpg >= 64) {
        int dummy = 0;
        minmax_cross<true>(mn, mx, dummy);
    }
}
__device__ __forceinline__ int grp_or(int v, int lpg) {
    if (lpg >= 2) v |= dppi<0xB1>(v);
    if (lpg >= 4) v |= dppi<0x4E>(v);
    if (lpg >= 8) v |= dppi<0x141>(v);
    if (lpg >= 16) v |= dppi<0x140>(v);
    unsigned a, b;
    if (lpg >= 32) { swap16((unsigned)v, a, b); v = (int)(a | b); }
    if (lpg >= 64) { swap32((unsigned)v, a, b); v = (int)(a | b); }
    return v;
}

__device__ __forceinline__ float grp_sum(float v, int lpg) {
    if (lpg >= 2) v = v + dppf<0xB1>(v);
    if (lpg >= 4) v = v + dppf<0x4E>(v);
    if (lpg >= 8) v = v + dppf<0x141>(v);
    if (lpg >= 16) v = v + dppf<0x140>(v);
    unsigned x, y;
    if (lpg >= 32) { swap16(ubits(v), x, y); v = fbits(x) + fbits(y); }   // own + partner, either order
    if (lpg >= 64) { swap32(ubits(v), x, y); v = fbits(x) + fbits(y); }
    return v;
}


// Canonical fp64 summation orders (oracle/awq_oracle.c ACT_*; include/awq_hip.h): two or
// three levels, so that a workgroup runs many short dependent chains instead of a few long
// ones (every level is still a fixed, ascending order: the bits do not depend on the launch)
constexpr int kRowBlock = 256;       // rows per column-sum block
constexpr int kRowSub = 32;          // rows per sub-block (a block = its sub-blocks' sums)
constexpr int kGroupBlock = 1024;    // groups per loss block
constexpr int kGroupSub = 64;        // groups per sub-block of a loss block
constexpr int kSuperBlocks = 32;     // loss blocks per super-block of a candidate's total

// 8 consecutive elements as fp32 (compute type of bf16 / fp16 / fp32 inputs)
template <int DT>
__device__ __forceinline__ void load8(const void* base, int64_t i, float (&v)[8]) {
    if (DT == AWQ_DTYPE_F32) {
        const float4* p = (const float4*)((const float*)base + i);
        const float4 a = p[0], b = p[1];
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
        v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
        const uint4 u = *(const uint4*)((const uint16_t*)base + i);
        const uint32_t h[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint16_t lo = (uint16_t)(h[j] & 0xFFFFu), hi = (uint16_t)(h[j] >> 16);
            if (DT == AWQ_DTYPE_BF16) {
                v[2 * j] = __uint_as_float((uint32_t)lo << 16);
                v[2 * j + 1] = __uint_as_float((uint32_t)hi << 16);
            } else {
                v[2 * j] = (float)__builtin_bit_cast(_Float16, lo);      // exact
                v[2 * j + 1] = (float)__builtin_bit_cast(_Float16, hi);
            }
        }
    }
}

// ---- column sums (canonical, fp64: rows ascending inside a 32-row sub-block, the
//      sub-blocks ascending inside a 256-row block) ----
// MODE 0, activations x [T, K]:  part0[b][k] = sum |x|,  part1[b][k] = sum x*x
// MODE 1, weights w [R, K]:      part0[b][k] = sum fp32(|w| / fp32(gmax[r, k/L] + 1e-6f))
// One lane per column and block; the sums are dependent fp64 chains, so the loads go out
// kColBatch rows ahead of them (a lane's loads are independent of its sums): the chain
// order is unchanged, only the memory latency overlaps.
constexpr int kColBatch = 16;
static_assert(kRowSub % kColBatch == 0, "a load batch stays inside one sub-block");

template <int DT, int MODE>
__global__ __launch_bounds__(256) void colsum_kernel(const void* __restrict__ src, int64_t rows, int64_t K,
                                                     int64_t L, const float* __restrict__ gmax,
                                                     double* __restrict__ part0, double* __restrict__ part1) {
    typedef Traits<DT> T;
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= K) return;
    const int64_t b = blockIdx.y;
    const int64_t r0 = b * kRowBlock;
    const int64_t r1 = (r0 + kRowBlock < rows) ? r0 + kRowBlock : rows;
    const typename T::S* p = (const typename T::S*)src;
    const int64_t G = K / L, gk = k / L;
    double s0 = 0.0, s1 = 0.0, u0 = 0.0, u1 = 0.0;
    for (int64_t r = r0; r < r1; r += kColBatch) {
        float v[kColBatch], den[kColBatch];
#pragma unroll
        for (int j = 0; j < kColBatch; ++j) {
            const int64_t rr = (r + j < r1) ? r + j : r1 - 1;   // in range; the tail is skipped below
            v[j] = T::load(p, rr * K + k);
            if (MODE == 1) den[j] = gmax[rr * G + gk] + 1e-6f;
        }
#pragma unroll
        for (int j = 0; j < kColBatch; ++j) {
            if (r + j < r1) {
                if (MODE == 0) {
                    const double d = (double)v[j];     // |x| and x*x are exact in fp64
                    u0 += __builtin_fabs(d);
                    u1 += d * d;
                } else {
                    u0 += (double)(__builtin_fabsf(v[j]) / den[j]);
                }
            }
        }
        if ((r + kColBatch - r0) % kRowSub == 0 || r + kColBatch >= r1) {   // a sub-block ends
            s0 += u0;
            s1 += u1;
            u0 = 0.0;
            u1 = 0.0;
        }
    }
    part0[b * K + k] = s0;
    if (MODE == 0) part1[b * K + k] = s1;
}

// out[k] = fp32(sum over blocks, ascending, fp64 / divisor)
__global__ __launch_bounds__(256) void colmean_kernel(const double* __restrict__ part, int64_t nblk, int64_t K,
                                                      double divisor, float* __restrict__ out) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= K) return;
    double s = 0.0;
    for (int64_t b = 0; b < nblk; b += kColBatch) {
        double v[kColBatch];
#pragma unroll
        for (int j = 0; j < kColBatch; ++j) v[j] = part[((b + j < nblk) ? b + j : nblk - 1) * K + k];
#pragma unroll
        for (int j = 0; j < kColBatch; ++j)
            if (b + j < nblk) s += v[j];
    }
    out[k] = (float)(s / divisor);
}

// Same sums, staged through LDS: a workgroup takes one 256-row block x kColTile columns;
// every thread loads 8-column octets of several rows (16-B loads, all in flight at once) and
// stores the fp32 terms (MODE 1: the quotient, computed at load time) in LDS; then
// kColTile lanes run the column chains (rows ascending, fp64) from LDS.  Needs K % 8 == 0
// and a 16-B aligned src.
// 32 columns: 32 KiB of LDS, several workgroups per CU overlap one another's load and chain
// phases (r90: 64 columns or a 128-column tile of raw 16-bit values were 5-25 % slower)
constexpr int kColTile = 32;
template <int DT, int MODE>
__global__ __launch_bounds__(256) void colsum_tile_kernel(const void* __restrict__ src, int64_t rows, int64_t K,
                                                          int64_t L, const float* __restrict__ gmax,
                                                          double* __restrict__ part0, double* __restrict__ part1) {
    __shared__ __attribute__((aligned(16))) float sv[kRowBlock][kColTile];
    const int tid = threadIdx.x;
    const int64_t kt = (int64_t)blockIdx.x * kColTile;
    const int64_t b = blockIdx.y, r0 = b * kRowBlock;
    const int nr = (int)((r0 + kRowBlock < rows) ? kRowBlock : rows - r0);
    constexpr int OPR = kColTile / 8, RPP = 256 / OPR;   // octets per row, rows per pass
    const int oc = tid % OPR, rl = tid / OPR;           // column octet, first row
    const int64_t k0 = kt + 8 * oc;
    const bool kin = k0 < K;
    constexpr int NI = kRowBlock / RPP;
    float v[NI][8];
    float den[NI];
#pragma unroll
    for (int it = 0; it < NI; ++it) {
        const int rr = rl + RPP * it;
        if (kin && rr < nr) {
            load8<DT>(src, (r0 + rr) * K + k0, v[it]);
            if (MODE == 1) den[it] = gmax[(r0 + rr) * (K / L) + k0 / L] + 1e-6f;
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[it][j] = 0.0f;
            if (MODE == 1) den[it] = 1.0f;
        }
    }
#pragma unroll
    for (int it = 0; it < NI; ++it) {
        const int rr = rl + RPP * it;
        if (MODE == 1)
#pragma unroll
            for (int j = 0; j < 8; ++j) v[it][j] = __builtin_fabsf(v[it][j]) / den[it];
        *(float4*)&sv[rr][8 * oc] = make_float4(v[it][0], v[it][1], v[it][2], v[it][3]);
        *(float4*)&sv[rr][8 * oc + 4] = make_float4(v[it][4], v[it][5], v[it][6], v[it][7]);
    }
    __syncthreads();
    // every thread: one column of one 32-row sub-block (rows ascending, fp64); then kColTile
    // lanes add the block's sub-block sums in order
    constexpr int NSUB = kRowBlock / kRowSub;
    static_assert(NSUB * kColTile == 256, "one sub-block chain per thread");
    const int col = tid % kColTile, sub = tid / kColTile;
    const int ra = sub * kRowSub, rb = min(ra + kRowSub, nr);
    double s0 = 0.0, s1 = 0.0;
    for (int r = ra; r < rb; r += 16) {
        float t[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) t[j] = sv[(r + j < rb) ? r + j : rb - 1][col];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if (r + j < rb) {
                const double d = (double)t[j];
                if (MODE == 0) {
                    s0 += __builtin_fabs(d);
                    s1 += d * d;
                } else {
                    s0 += d;
                }
            }
        }
    }
    __shared__ double ss0[NSUB][kColTile], ss1[NSUB][kColTile];
    ss0[sub][col] = s0;
    if (MODE == 0) ss1[sub][col] = s1;
    __syncthreads();
    if (tid >= kColTile || kt + tid >= K) return;
    double a0 = 0.0, a1 = 0.0;
    for (int u = 0; u < NSUB && u * kRowSub < nr; ++u) {   // non-empty sub-blocks, ascending
        a0 += ss0[u][tid];
        if (MODE == 0) a1 += ss1[u][tid];
    }
    part0[b * K + kt + tid] = a0;
    if (MODE == 0) part1[b * K + kt + tid] = a1;
}

// Lane layout shared by the group kernels: LPG = L / 8 lanes per group (8 consecutive
// elements per lane), GPW = 64 / LPG groups per wave, the wave's groups are GPW
// consecutive ROWS of one group column g (the same k range: table / x_sq loads are shared).
struct GroupLane {
    int64_t r, g, k0;
    bool valid;
};

// (EPL elements per lane: 8, or 16 = two consecutive 8-element chunks)
template <int EPL = 8>
__device__ __forceinline__ bool group_lane(int64_t item, int64_t R, int64_t G, int lpg, GroupLane& gl) {
    const int lane = threadIdx.x & 63;
    const int gpw = 64 / lpg;
    const int64_t nrb = (R + gpw - 1) / gpw;
    if (item >= nrb * G) return false;
    gl.g = item / nrb;
    const int64_t rb = item - gl.g * nrb;
    gl.r = rb * gpw + lane / lpg;
    gl.valid = gl.r < R;
    gl.k0 = gl.g * (int64_t)(EPL * lpg) + EPL * (lane % lpg);
    return true;
}

// awq_weight_colsum in ONE pass over W for group sizes 32 / 64 / 128 / 256 (K % gs == 0, 16-B
// aligned): a workgroup takes one 256-row block x one group column (gs columns), in stages of
// RS = 8192 / gs rows (32 KiB of fp32 terms in LDS): every thread loads 4 octets of the stage
// (all in flight), the gs / 8 threads of a row reduce its group's NaN-propagating max |w|
// (as group_absmax_kernel), and store fp32(|w| / fp32(gmax + 1e-6f)) into LDS; then, with the
// next stage's loads in flight, each of the 256 threads runs one (column, 32-row sub-block)
// chain of the stage in fp64, rows
// ascending, and the sub-block sums are added ascending per column at the end — the
// canonical order of colsum_kernel, so part[] is bit-identical, with W read once instead of
// twice (round 5).  (A/B builds: -DAWQ_WMEAN_FUSED=0 keeps the two-pass path.)
#ifndef AWQ_WMEAN_FUSED
#define AWQ_WMEAN_FUSED 1
#endif
template <int DT, int GS>
__global__ __launch_bounds__(256) void wcolsum_fused_kernel(const void* __restrict__ w, int64_t rows, int64_t K,
                                                            double* __restrict__ part) {
    constexpr int RS = 8192 / GS;                // rows per stage
    constexpr int OPR = GS / 8;                  // octets (threads) per row
    constexpr int RPP = 256 / OPR;               // rows per load pass
    constexpr int NP = RS / RPP;                 // load passes per stage (4)
    constexpr int SBS = RS / kRowSub;            // sub-blocks per stage
    constexpr int NSB = kRowBlock / kRowSub;     // sub-blocks per block (8)
    static_assert(NP * RPP == RS && SBS * GS == 256, "one chain per thread per stage");
    __shared__ __attribute__((aligned(16))) float sv[RS][GS];
    __shared__ double ssum[NSB][GS];
    const int tid = threadIdx.x;
    const int64_t kt = (int64_t)blockIdx.x * GS;
    const int64_t b = blockIdx.y, r0 = b * kRowBlock;
    const int nr = (int)((r0 + kRowBlock < rows) ? kRowBlock : rows - r0);
    const int oc = tid % OPR, rl = tid / OPR;
    const int c = tid % GS, sbl = tid / GS;      // this thread's chain: column, sub-block of the stage
    float v[NP][8];
    auto load_stage = [&](int st) {
#pragma unroll
        for (int it = 0; it < NP; ++it) {
            const int rr = st * RS + rl + RPP * it;
            if (rr < nr) load8<DT>(w, (r0 + rr) * K + kt + 8 * oc, v[it]);
            else for (int j = 0; j < 8; ++j) v[it][j] = 0.0f;
        }
    };
    load_stage(0);
    for (int st = 0; st * RS < nr; ++st) {
#pragma unroll
        for (int it = 0; it < NP; ++it) {
            float m = 0.0f, dummy = 0.0f;
            int nan = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float a = __builtin_fabsf(v[it][j]);
                nan |= a != a;
                m = a > m ? a : m;
            }
            grp_minmax(dummy, m, nan, OPR);
            const float den = (nan ? __builtin_nanf("") : m) + 1e-6f;
            const int rr = rl + RPP * it;
#pragma unroll
            for (int j = 0; j < 8; ++j) v[it][j] = __builtin_fabsf(v[it][j]) / den;
            *(float4*)&sv[rr][8 * oc] = make_float4(v[it][0], v[it][1], v[it][2], v[it][3]);
            *(float4*)&sv[rr][8 * oc + 4] = make_float4(v[it][4], v[it][5], v[it][6], v[it][7]);
        }
        __syncthreads();
        if ((st + 1) * RS < nr) load_stage(st + 1);   // next stage's loads in flight during the chains
        const int sb = st * SBS + sbl;           // sub-block in the block
        const int ra = sbl * kRowSub, rb = min(ra + kRowSub, nr - st * RS);
        if (ra < rb) {
            double u = 0.0;
            for (int r = ra; r < rb; ++r) u += (double)sv[r][c];
            ssum[sb][c] = u;
        }
        __syncthreads();
    }
    if (tid >= GS) return;
    double a = 0.0;
    for (int u = 0; u < NSB && u * kRowSub < nr; ++u) a += ssum[u][tid];   // non-empty sub-blocks, ascending
    part[b * K + kt + tid] = a;
}

// NaN-propagating max |w| of every group (awq_weight_mean's normaliser)
template <int DT>
__global__ __launch_bounds__(256) void group_absmax_kernel(const void* __restrict__ w, int64_t R, int64_t K,
                                                           int lpg, float* __restrict__ gmax) {
    const int64_t G = K / (8 * lpg);
    const int64_t nw = (int64_t)gridDim.x * 4;
    for (int64_t item = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);; item += nw) {
        GroupLane gl;
        if (!group_lane(item, R, G, lpg, gl)) break;
        float v[8];
        if (gl.valid) load8<DT>(w, gl.r * K + gl.k0, v);
        else for (int j = 0; j < 8; ++j) v[j] = 0.0f;
        float m = 0.0f;
        int nan = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float a = __builtin_fabsf(v[j]);
            nan |= a != a;
            m = a > m ? a : m;
        }
        for (int o = 1; o < lpg; o <<= 1) {
            const float t = __shfl_xor(m, o, 64);
            m = t > m ? t : m;
            nan |= __shfl_xor(nan, o, 64);
        }
        if (gl.valid && (threadIdx.x & 63) % lpg == 0) gmax[gl.r * G + gl.g] = nan ? __builtin_nanf("") : m;
    }
}

// ---- the table's power function (include/awq_hip.h awq_act_scale_table: "awq_pow") ----
// x^r from IEEE fp64 +, *, /, fma and rint only, in one fixed order, so that every
// implementation of the definition (this kernel, oracle_act_scale_table) gets the same bits;
// a libm pow differs between math libraries in the last ulp.  ~1e-16 relative accuracy.
namespace detpow {
constexpr double kLn2Hi = 6.93147180369123816490e-01;   // 0x3FE62E42FEE00000: e * kLn2Hi exact
constexpr double kLn2Lo = 1.90821492927058770002e-10;
constexpr double kInvLn2 = 1.44269504088896338700e+00;

__device__ __forceinline__ double two_pow(int n) {       // 2^n, -1022 <= n <= 1023
    return __longlong_as_double((long long)(n + 1023) << 52);
}

// ln x, x positive finite: x = m 2^e with m in [sqrt(2)/2, sqrt(2)), f = (m - 1) / (m + 1),
// ln m = 2f + 2f f^2 P(f^2), P = sum_{j=1..12} f^(2j-2) / (2j + 1) by Horner
__device__ double log_p(double x) {
#pragma clang fp contract(off)
    int e = 0;
    if (x < 0x1p-1022) { x = x * 0x1p54; e = -54; }            // subnormal: exact rescale
    const unsigned long long u = (unsigned long long)__double_as_longlong(x);
    e += (int)((u >> 52) & 0x7FF) - 1023;
    double m = __longlong_as_double((long long)((u & 0xFFFFFFFFFFFFFull) | 0x3FF0000000000000ull));  // [1, 2)
    if (m > 1.4142135623730951) { m = m * 0.5; e += 1; }
    const double f = (m - 1.0) / (m + 1.0);
    const double f2 = f * f;
    double p = 1.0 / 25.0;
    for (int j = 11; j >= 1; --j) p = __builtin_fma(p, f2, 1.0 / (double)(2 * j + 1));
    const double t = 2.0 * f;
    const double lm = __builtin_fma(t * f2, p, t);
    const double de = (double)e;
    return __builtin_fma(de, kLn2Hi, __builtin_fma(de, kLn2Lo, lm));
}

// e^y: k = rint(y / ln 2), t = y - k ln 2 (two fma), e^t = 1 + t(1 + t/2(1 + ... (1 + t/15))),
// times 2^k (two steps below 2^-1022: one rounding, into the subnormals)
__device__ double exp_p(double y) {
#pragma clang fp contract(off)
    if (y != y) return y;
    if (y > 709.8) return __builtin_inf();
    if (y < -746.0) return 0.0;
    const double k = __builtin_rint(y * kInvLn2);
    double t = __builtin_fma(-k, kLn2Hi, y);
    t = __builtin_fma(-k, kLn2Lo, t);
    double p = 1.0;
    for (int j = 15; j >= 1; --j) p = __builtin_fma(p, t / (double)j, 1.0);
    const int ki = (int)k;
    if (ki > 1023) return (p * two_pow(1023)) * two_pow(ki - 1023);
    if (ki < -1022) return (p * two_pow(ki + 600)) * two_pow(-600);
    return p * two_pow(ki);
}

// x^r for x >= 0 (a statistic), r in [0, 1]: C99 pow on the special values
__device__ double pow_p(double x, double r) {
#pragma clang fp contract(off)
    if (r == 0.0) return 1.0;
    if (x != x || x < 0.0) return __builtin_nan("");
    if (x == 0.0) return 0.0;
    if (__builtin_isinf(x)) return x;
    return exp_p(r * log_p(x));
}
}  // namespace detpow

// candidate i's raw scale of channel k (fp64): x_mean^r [/ (w_mean^(1-r) + 1e-4)], >= 1e-4
__device__ __forceinline__ double raw_scale(const float* x_mean, const float* w_mean, int64_t k, double r) {
    double s = detpow::pow_p((double)x_mean[k], r);
    if (w_mean) s = s / (detpow::pow_p((double)w_mean[k], 1.0 - r) + 1e-4);
    return s < 1e-4 ? 1e-4 : s;   // NaN stays NaN
}

// table[i][k] = fp32(raw / sqrt(max_k raw * min_k raw)), inf / NaN -> 1; one workgroup per
// candidate; max / min propagate NaN (order-independent, so any reduction order is exact)
// (16 waves per workgroup: the fp64 pow chains are latency-bound, one workgroup per CU)
constexpr int kTableThreads = 1024;
__global__ __launch_bounds__(kTableThreads) void scale_table_kernel(const float* __restrict__ x_mean,
                                                          const float* __restrict__ w_mean, int64_t K, int n_grid,
                                                          float* __restrict__ table) {
    __shared__ double smx[kTableThreads], smn[kTableThreads];
    __shared__ int snan[kTableThreads];
    const int i = blockIdx.x, tid = threadIdx.x;
    const double r = (double)i / (double)n_grid;
    double mx = -__builtin_inf(), mn = __builtin_inf();
    int nan = 0;
    for (int64_t k = tid; k < K; k += kTableThreads) {
        const double s = raw_scale(x_mean, w_mean, k, r);
        if (s != s) nan = 1;
        mx = s > mx ? s : mx;
        mn = s < mn ? s : mn;
    }
    smx[tid] = mx;
    smn[tid] = mn;
    snan[tid] = nan;
    __syncthreads();
    for (int o = kTableThreads / 2; o > 0; o >>= 1) {
        if (tid < o) {
            smx[tid] = smx[tid + o] > smx[tid] ? smx[tid + o] : smx[tid];
            smn[tid] = smn[tid + o] < smn[tid] ? smn[tid + o] : smn[tid];
            snan[tid] |= snan[tid + o];
        }
        __syncthreads();
    }
    const double norm = snan[0] ? __builtin_nan("") : sqrt(smx[0] * smn[0]);
    // this workgroup's slice of the row (blockIdx.y of gridDim.y: every slice's workgroup
    // finds the same max / min, so the row's normaliser is the same in all of them)
    const int64_t per = (K + gridDim.y - 1) / gridDim.y;
    const int64_t k0 = (int64_t)blockIdx.y * per, k1 = (k0 + per < K) ? k0 + per : K;
    for (int64_t k = k0 + tid; k < k1; k += kTableThreads) {
        double s = raw_scale(x_mean, w_mean, k, r) / norm;
        if (s != s || __builtin_isinf(s)) s = 1.0;
        table[(int64_t)i * K + k] = (float)s;
    }
}

// awq_act_scale_table_ws: the same table with every power evaluated once (round 5).  Pass 1:
// thread (slice, k) of candidate blockIdx.y keeps raw_scale in work and its 256-channel
// slice's NaN-skipping max / min and NaN flag go to part; pass 2: every workgroup folds its
// candidate's slice partials (max / min are order-independent) into the normaliser and
// writes its slice.  Same values as scale_table_kernel, which recomputes pass 1 per slice.
constexpr int kTabSlice = 256;
__global__ __launch_bounds__(kTabSlice) void table_raw_kernel(const float* __restrict__ x_mean,
                                                              const float* __restrict__ w_mean, int64_t K, int n_grid,
                                                              double* __restrict__ raw, double* __restrict__ part) {
    __shared__ double smx[kTabSlice], smn[kTabSlice];
    __shared__ int snan[kTabSlice];
    const int i = blockIdx.y, tid = threadIdx.x;
    const int64_t k = (int64_t)blockIdx.x * kTabSlice + tid;
    const double r = (double)i / (double)n_grid;
    double mx = -__builtin_inf(), mn = __builtin_inf();
    int nan = 0;
    if (k < K) {
        const double s = raw_scale(x_mean, w_mean, k, r);
        raw[(int64_t)i * K + k] = s;
        if (s != s) nan = 1;
        mx = s > mx ? s : mx;
        mn = s < mn ? s : mn;
    }
    smx[tid] = mx;
    smn[tid] = mn;
    snan[tid] = nan;
    __syncthreads();
    for (int o = kTabSlice / 2; o > 0; o >>= 1) {
        if (tid < o) {
            smx[tid] = smx[tid + o] > smx[tid] ? smx[tid + o] : smx[tid];
            smn[tid] = smn[tid + o] < smn[tid] ? smn[tid + o] : smn[tid];
            snan[tid] |= snan[tid + o];
        }
        __syncthreads();
    }
    if (tid == 0) {
        double* q = part + ((int64_t)i * gridDim.x + blockIdx.x) * 3;
        q[0] = smx[0];
        q[1] = smn[0];
        q[2] = (double)snan[0];
    }
}
__global__ __launch_bounds__(kTabSlice) void table_norm_kernel(const double* __restrict__ raw,
                                                               const double* __restrict__ part, int64_t K,
                                                               float* __restrict__ table) {
    __shared__ double smx[kTabSlice], smn[kTabSlice];
    __shared__ int snan[kTabSlice];
    const int i = blockIdx.y, tid = threadIdx.x;
    const int S = (int)gridDim.x;
    double mx = -__builtin_inf(), mn = __builtin_inf();
    int nan = 0;
    for (int q = tid; q < S; q += kTabSlice) {
        const double* p = part + ((int64_t)i * S + q) * 3;
        mx = p[0] > mx ? p[0] : mx;
        mn = p[1] < mn ? p[1] : mn;
        nan |= p[2] != 0.0;
    }
    smx[tid] = mx;
    smn[tid] = mn;
    snan[tid] = nan;
    __syncthreads();
    for (int o = kTabSlice / 2; o > 0; o >>= 1) {
        if (tid < o) {
            smx[tid] = smx[tid + o] > smx[tid] ? smx[tid + o] : smx[tid];
            smn[tid] = smn[tid + o] < smn[tid] ? smn[tid + o] : smn[tid];
            snan[tid] |= snan[tid + o];
        }
        __syncthreads();
    }
    const double norm = snan[0] ? __builtin_nan("") : sqrt(smx[0] * smn[0]);
    const int64_t k = (int64_t)blockIdx.x * kTabSlice + tid;
    if (k >= K) return;
    double s = raw[(int64_t)i * K + k] / norm;
    if (s != s || __builtin_isinf(s)) s = 1.0;
    table[(int64_t)i * K + k] = (float)s;
}

// Per group and candidate i: w' = RN(w * s_i), RTN parameters of w' (awq.py:173-213),
// q (awq.py:245-248), the reference's dequantize dq = fp16(fp16(q - z) * fp16(scale))
// (awq.py:459-539), ŵ = dq / s_i (fp32), e = ŵ - w, loss = sum x_sq[k] * (e * e): each
// lane sums its 8 elements in order, then the xor-butterfly (pairwise) tree over the
// group's LPG lanes; part[i * stride + r * G + g] (fp32).
// ŵ = RN_f32(dq / s) from rs = RN_f32(1 / s) with one Markstein correction: exact for every
// fp16-valued dq and every s in [2^-60, 2^60] (awq_selftest 1: all 2^23 mantissas of s x
// every positive finite fp16 dq, 2.7e11 pairs, against the IEEE division; the steps are
// scale-invariant while no intermediate leaves the normal range, which this s range keeps)
__device__ __forceinline__ float mquot(float a, float s, float rs) {
    const float q0 = a * rs;
    const float r = __builtin_fmaf(-s, q0, a);
    return __builtin_fmaf(r, rs, q0);
}
// the same with a = the low (HI = false) or high half of a packed fp16 pair: the two products
// with a read the fp16 value directly (v_fma_mix_f32; q0 = a * rs + (-0): the product's bits,
// signed zeros included), the bits of mquot((float)a, s, rs)
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
template <bool HI>
__device__ __forceinline__ float mquot_h(h2v a, float s, float rs) {
    float q0, r;
    const float nz = -0.0f;
    if (HI) {
        asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(q0) : "v"(a), "v"(rs), "v"(nz));
        asm("v_fma_mix_f32 %0, -%1, %2, %3 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "=v"(r) : "v"(s), "v"(q0), "v"(a));
    } else {
        asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(q0) : "v"(a), "v"(rs), "v"(nz));
        asm("v_fma_mix_f32 %0, -%1, %2, %3 op_sel_hi:[0,0,1]" : "=v"(r) : "v"(s), "v"(q0), "v"(a));
    }
    return __builtin_fmaf(r, rs, q0);
}

// RN_f32(a * r) with a = the low / high fp16 half (v_fma_mix_f32 with a -0 addend: the product's
// bits, signed zeros included)
template <bool HI>
__device__ __forceinline__ float mprod_h(h2v a, float r) {
    float p;
    const float nz = -0.0f;
    if (HI) asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(p) : "v"(a), "v"(r), "v"(nz));
    else asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(p) : "v"(a), "v"(r), "v"(nz));
    return p;
}

// LPG: lanes per group as a constant (0 = the run-time lpg argument); SYM: symmetric;
// EPL: elements per lane — 16 (two consecutive 8-element chunks, LPG = gs / 16 lanes per
// group) halves the per-candidate group work per element (reductions, RTN parameters, table
// checks).  The loss tree is unchanged: each chunk is summed in order, the lane adds its two
// chunks (the tree's first pairwise level; + is commutative), grp_sum does the rest.
// (A/B builds: -DAWQ_ACT_LDS=0 restores round 4's per-candidate register loads of the tables)
#ifndef AWQ_ACT_LDS
#define AWQ_ACT_LDS 1
#endif
// Round-6 trims of the loss kernel's per-element work (A/B builds: = 0 restores round 5's):
//   AWQ_ACT_NAN_HOIST   the weights' NaN flag once per item, not per candidate and element
//                       (RN(w * s) is NaN exactly when w is: s is a positive finite table entry)
//   AWQ_ACT_NAN_RTABLE  out-of-range reciprocals as NaN: the Markstein path runs unchecked and a
//                       wave whose loss came out NaN redoes the candidate with IEEE divisions
//                       (no per-candidate min over the lane's reciprocals)
//   AWQ_ACT_MIX_DQ      dq kept as packed fp16 pairs, fed to v_fma_mix_f32 in the Markstein
//                       quotient (no fp16 -> f32 widening per element)
#ifndef AWQ_ACT_NAN_HOIST
#define AWQ_ACT_NAN_HOIST 1
#endif
#ifndef AWQ_ACT_NAN_RTABLE
#define AWQ_ACT_NAN_RTABLE 1
#endif
#ifndef AWQ_ACT_MIX_DQ
#define AWQ_ACT_MIX_DQ 1
#endif
//   AWQ_ACT_F16_TAIL    (round 6, later) bf16 / fp16 weights: rint, clamp and the fp16 product in
//                       packed fp16 (two elements per instruction)
#ifndef AWQ_ACT_F16_TAIL
#define AWQ_ACT_F16_TAIL 1
#endif
//   AWQ_ACT_F16_PLAIN   fp16 weights, a wave whose group scales are all < 14: the plain quotient
#ifndef AWQ_ACT_F16_PLAIN
#define AWQ_ACT_F16_PLAIN 1
#endif
//   AWQ_ACT_F16_PACKED  fp16 weights: w' kept as packed fp16 pairs (min / max, the quotient's
//                       operand), t and t + z in packed fp16
#ifndef AWQ_ACT_F16_PACKED
#define AWQ_ACT_F16_PACKED 1
#endif
//   AWQ_ACT_PK_F32      bf16 weights: w s, w' r and t + z as v_pk_mul_f32 / v_pk_add_f32 pairs
#ifndef AWQ_ACT_PK_F32
#define AWQ_ACT_PK_F32 1
#endif
// The table ring's waits are explicit: the compiler's own wait before an LDS read that may
// alias an LDS-DMA covers every DMA in flight (vmcnt(0)), which would serialise the prefetch,
// so the ring is read by inline-asm ds_read_b128 it does not track, with explicit lgkmcnt
// waits; vm_wait<N> = s_waitcnt vmcnt(N) (all but the wave's N youngest vector-memory
// operations done; loads, stores and LDS-DMA count together in issue order).
template <int N>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ uint32_t lds_addr(const float* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)p;
}
typedef float f4v __attribute__((ext_vector_type(4)));
template <int OFF>
__device__ __forceinline__ f4v lds_read4(uint32_t a) {
    f4v t;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(t) : "v"(a), "n"(OFF) : "memory");
    return t;
}
// A ring slot's 2 * EPL floats: EPL scale-table entries at a (into s, waited for here) and
// EPL reciprocals at a + 4 GSZ (left in flight in rp until lds_slot_rs).  The lgkmcnt waits
// take the loaded registers as operands, so no use of them can be scheduled above the wait;
// LDS reads complete in order, so lgkmcnt(EPL / 4) means the scale reads are done.
template <int EPL, int GSZ>
__device__ __forceinline__ void lds_slot_s(uint32_t a, float (&s)[EPL], f4v (&rp)[EPL / 4]) {
    static_assert(EPL == 8 || EPL == 16, "8 or 16 elements per lane");
    f4v t[EPL / 4];
    t[0] = lds_read4<0>(a);
    t[1] = lds_read4<16>(a);
    if constexpr (EPL == 16) {
        t[2] = lds_read4<32>(a);
        t[3] = lds_read4<48>(a);
    }
    rp[0] = lds_read4<4 * GSZ>(a);
    rp[1] = lds_read4<4 * GSZ + 16>(a);
    if constexpr (EPL == 16) {
        rp[2] = lds_read4<4 * GSZ + 32>(a);
        rp[3] = lds_read4<4 * GSZ + 48>(a);
        asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]) : : "memory");
    } else {
        asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(t[0]), "+v"(t[1]) : : "memory");
    }
#pragma unroll
    for (int q = 0; q < EPL / 4; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) s[4 * q + e] = t[q][e];
}
// EPL 16 with AWQ_ACT_RS_PAIRS: the reciprocals read as (j, j + 8) pairs by ds_read2_b32 — the
// register pairs the loss's packed ops want (the two 8-element chunks go through v_pk_fma_f32 /
// v_pk_add_f32 side by side), instead of four ds_read_b128 and a v_mov per element to re-pair them
#ifndef AWQ_ACT_RS_PAIRS
#define AWQ_ACT_RS_PAIRS 1
#endif
template <int O0, int O1>
__device__ __forceinline__ f2 lds_read2(uint32_t a) {
    f2 t;
    asm volatile("ds_read2_b32 %0, %1 offset0:%2 offset1:%3" : "=v"(t) : "v"(a), "n"(O0), "n"(O1) : "memory");
    return t;
}
template <int GSZ>
__device__ __forceinline__ void lds_slot_s_pairs(uint32_t a, float (&s)[16], f2 (&rq)[8]) {
    f4v t[4];
    t[0] = lds_read4<0>(a);
    t[1] = lds_read4<16>(a);
    t[2] = lds_read4<32>(a);
    t[3] = lds_read4<48>(a);
    const uint32_t b = a + 4 * GSZ;                      // the reciprocal row (dword offsets <= 15)
    rq[0] = lds_read2<0, 8>(b);
    rq[1] = lds_read2<1, 9>(b);
    rq[2] = lds_read2<2, 10>(b);
    rq[3] = lds_read2<3, 11>(b);
    rq[4] = lds_read2<4, 12>(b);
    rq[5] = lds_read2<5, 13>(b);
    rq[6] = lds_read2<6, 14>(b);
    rq[7] = lds_read2<7, 15>(b);
    asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]) : : "memory");
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) s[4 * q + e] = t[q][e];
}
__device__ __forceinline__ void lds_slot_rs_pairs(f2 (&rq)[8], float (&rs)[16]) {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(rq[0]), "+v"(rq[1]), "+v"(rq[2]), "+v"(rq[3]), "+v"(rq[4]), "+v"(rq[5]), "+v"(rq[6]), "+v"(rq[7])
                 :
                 : "memory");
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        rs[k] = rq[k].x;
        rs[k + 8] = rq[k].y;
    }
}

template <int EPL>
__device__ __forceinline__ void lds_slot_rs(f4v (&rp)[EPL / 4], float (&rs)[EPL]) {
    if constexpr (EPL == 16)
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(rp[0]), "+v"(rp[1]), "+v"(rp[2]), "+v"(rp[3]) : : "memory");
    else
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(rp[0]), "+v"(rp[1]) : : "memory");
#pragma unroll
    for (int q = 0; q < EPL / 4; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) rs[4 * q + e] = rp[q][e];
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t act_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

template <int DT, int LPG, bool SYM, int EPL>
__global__ __launch_bounds__(256, 3) void act_loss_kernel(const void* __restrict__ w, int64_t R, int64_t K, int lpg_rt,
                                                       int qmin, int qmax, const float* __restrict__ table,
                                                       const float* __restrict__ rtable, int n_grid,
                                                       const float* __restrict__ x_sq, float* __restrict__ part,
                                                       int64_t stride) {
    typedef HwFmt<DT> H;
    constexpr bool kF16Packed = DT == AWQ_DTYPE_F16 && AWQ_ACT_F16_PACKED && AWQ_ACT_F16_TAIL && AWQ_ACT_MIX_DQ &&
                                AWQ_ACT_NAN_HOIST;
    const int lpg = LPG ? LPG : lpg_rt;
    constexpr int sym = SYM ? 1 : 0;
    const int64_t G = K / (EPL * lpg);
    const int64_t nw = (int64_t)gridDim.x * 4;
    const bool leader = (threadIdx.x & 63) % lpg == 0;
    const float rq = 1.0f / (float)(qmax - qmin);   // RN_f32(1 / 15) or RN_f32(1 / 255)
    // Compile-time group sizes: each candidate's [scale row | reciprocal row] slice of the
    // wave's group column (8 B per element) comes in by LDS-DMA one candidate ahead, into a
    // two-slot ring per wave — no VGPRs held for the prefetch (register prefetch cost a wave
    // of occupancy and lost 9-12 %, round 5 r5h; this ring: bf16 -4 %, fp16 +-0, r5n).  Per
    // candidate i: wait for slot i & 1 (vmcnt(1): only candidate i - 1's loss store may still
    // be in flight — the store is a buffer store every lane issues, so the count is exact),
    // read it, issue candidate i + 1's DMA into the other slot, compute, store.
#if AWQ_ACT_LDS
    constexpr bool kLds = LPG > 0;
#else
    constexpr bool kLds = false;
#endif
    constexpr int GSZ = (LPG > 0 ? LPG : 1) * EPL;                   // group size
    constexpr int NQ = GSZ * 8 / 1024 > 0 ? GSZ * 8 / 1024 : 1;     // DMAs per candidate
    __shared__ __attribute__((aligned(16))) float ring[kLds ? 4 * 2 * 2 * GSZ : 1];
    float* const wr = ring + (kLds ? (threadIdx.x >> 6) * 2 * 2 * GSZ : 0);
    const int lane = threadIdx.x & 63;
    const float* const rt = rtable ? rtable : table;   // (no reciprocal table: that half is unread)
    auto dma = [&](int64_t g, int cand, int slot) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int e = q * 256 + 4 * lane;   // float index in [scale row | reciprocal row]
            if (e < 2 * GSZ) {
                const float* src = e < GSZ ? table + (int64_t)cand * K + g * GSZ + e
                                           : rt + (int64_t)cand * K + g * GSZ + (e - GSZ);
                __builtin_amdgcn_global_load_lds(
                    src, (__attribute__((address_space(3))) void*)(wr + slot * 2 * GSZ + q * 256), 16, 0, 0);
            }
        }
        asm volatile("" ::: "memory");   // the loss store stays younger than this DMA (vmcnt(1))
    };
    for (int64_t item = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);; item += nw) {
        GroupLane gl;
        if (!group_lane<EPL>(item, R, G, lpg, gl)) break;
        if constexpr (kLds) vm_wait<0>();   // the previous item's last DMA has landed in its slot
        float v[EPL], h[EPL];
#pragma unroll
        for (int c = 0; c < EPL; c += 8) {
            if (gl.valid) load8<DT>(w, gl.r * K + gl.k0 + c, *(float(*)[8]) & v[c]);
            else for (int j = 0; j < 8; ++j) v[c + j] = 0.0f;
            load8<AWQ_DTYPE_F32>(x_sq, gl.k0 + c, *(float(*)[8]) & h[c]);
        }
        if constexpr (kLds) dma(gl.g, 0, 0);
        const float* const cw = wr + (lane % lpg) * EPL;   // this lane's elements in a ring slot
#if AWQ_ACT_NAN_HOIST
        int nan_w = 0;                                      // the group's weights hold a NaN
#pragma unroll
        for (int j = 0; j < EPL; ++j) nan_w |= v[j] != v[j];
        nan_w = grp_or(nan_w, lpg);
#endif
        for (int i = 0; i < n_grid; ++i) {
            float s[EPL], ws[EPL];
            float rs[EPL];
            f4v rp[EPL / 4];
            [[maybe_unused]] f2 rsp[8];   // (j, j + 8) reciprocal pairs
            constexpr bool kPairs = EPL == 16 && AWQ_ACT_RS_PAIRS;
            if constexpr (kLds) {
                // slot i & 1 holds candidate i once every operation but the previous
                // candidate's store is done (i = 0: the item's loads and first DMA)
                if (i == 0) vm_wait<0>();
                else vm_wait<1>();
                if constexpr (kPairs)
                    lds_slot_s_pairs<GSZ>(lds_addr(cw + (i & 1) * 2 * GSZ), *(float(*)[16]) & s, rsp);
                else
                    lds_slot_s<EPL, GSZ>(lds_addr(cw + (i & 1) * 2 * GSZ), s, rp);   // (rp unused without rtable)
                dma(gl.g, i + 1 < n_grid ? i + 1 : i, (i + 1) & 1);   // (last: a harmless reload)
            } else {
#pragma unroll
                for (int c = 0; c < EPL; c += 8) load8<AWQ_DTYPE_F32>(table, (int64_t)i * K + gl.k0 + c, *(float(*)[8]) & s[c]);
            }
            // min / max skipping NaN (fmin / fmax; the signs of zero extrema cannot change the
            // scale or zero point) with NaN tracked on the side: torch's NaN-propagating
            // min / max once combined
            float mn = __builtin_inff(), mx = -__builtin_inff();
#if AWQ_ACT_NAN_HOIST
            const int nan = nan_w;
            [[maybe_unused]] h2v wsp[EPL / 2];   // fp16 weights: w' as packed fp16 pairs
            if constexpr (kF16Packed) {
                // RN_f16(RN_f32(w s)) two at a time (v_cvt_pk_f16_f32), min / max as v_pk_min_f16 /
                // v_pk_max_f16 (NaN skipped like fminf / fmaxf; NaN is tracked by nan_w)
#pragma unroll
                for (int j = 0; j < EPL; j += 2)
                    wsp[j / 2] = __builtin_convertvector((f2){opq(v[j] * s[j]), opq(v[j + 1] * s[j + 1])}, h2v);
                h2v a = wsp[0], b = wsp[0];
#pragma unroll
                for (int k = 1; k < EPL / 2; ++k) {
                    a = __builtin_elementwise_min(a, wsp[k]);
                    b = __builtin_elementwise_max(b, wsp[k]);
                }
                mn = __builtin_fminf((float)a.x, (float)a.y);
                mx = __builtin_fmaxf((float)b.x, (float)b.y);
#pragma unroll
                for (int j = 0; j < EPL; ++j) ws[j] = (float)wsp[j / 2][j & 1];   // (rare paths only)
            } else if constexpr (DT == AWQ_DTYPE_BF16 && AWQ_ACT_PK_F32 >= 2) {
                // the products two at a time (v_pk_mul_f32: the same IEEE ops in one instruction)
#pragma unroll
                for (int j = 0; j < EPL; j += 2) {
                    const f2 p = (f2){v[j], v[j + 1]} * (f2){s[j], s[j + 1]};
                    ws[j] = H::rn(p.x);
                    ws[j + 1] = H::rn(p.y);
                }
#pragma unroll
                for (int j = 0; j < EPL; ++j) {
                    mn = __builtin_fminf(mn, ws[j]);
                    mx = __builtin_fmaxf(mx, ws[j]);
                }
            } else {
#pragma unroll
                for (int j = 0; j < EPL; ++j) {
                    ws[j] = H::rn(v[j] * s[j]);
                    mn = __builtin_fminf(mn, ws[j]);
                    mx = __builtin_fmaxf(mx, ws[j]);
                }
            }
            grp_minmax_nn(mn, mx, lpg);
#else
            int nan = 0;
#pragma unroll
            for (int j = 0; j < EPL; ++j) {
                ws[j] = H::rn(v[j] * s[j]);
                nan |= ws[j] != ws[j];
                mn = __builtin_fminf(mn, ws[j]);
                mx = __builtin_fmaxf(mx, ws[j]);
            }
            grp_minmax(mn, mx, nan, lpg);
#endif
            if (nan) { mn = __builtin_nanf(""); mx = __builtin_nanf(""); }
            float cs, cz, r;
            hw_group_params<DT>(mn, mx, nan, qmin, qmax, sym, rq, cs, cz, r);
            float acc[EPL / 8];
#pragma unroll
            for (int c = 0; c < EPL / 8; ++c) acc[c] = 0.0f;
            // channel reciprocals for ŵ = dq / s (0 = outside the proven range: IEEE division)
            bool mq = false;
            // (the ring's reciprocal reads are waited for with or without a reciprocal table:
            //  registers an asm load is still writing must not be reused)
            if constexpr (kLds) {
                if constexpr (kPairs) lds_slot_rs_pairs(rsp, *(float(*)[16]) & rs);
                else lds_slot_rs<EPL>(rp, rs);
            }
            if (rtable != nullptr) {
                if constexpr (!kLds) {
#pragma unroll
                    for (int c = 0; c < EPL; c += 8)
                        load8<AWQ_DTYPE_F32>(rtable, (int64_t)i * K + gl.k0 + c, *(float(*)[8]) & rs[c]);
                }
#if AWQ_ACT_NAN_RTABLE
                mq = true;            // out-of-range entries are NaN: checked on the losses below
#else
                float m = rs[0];
#pragma unroll
                for (int j = 1; j < EPL; ++j) m = __builtin_fminf(m, rs[j]);
                mq = __builtin_amdgcn_ballot_w64(!(m > 0.0f)) == 0;   // wave-uniform
#endif
            }
            if (cs > 0.0f && cs < __builtin_inff()) {
                // finite positive scale (every group but constant fp16 / inf / NaN ones):
                // RN(w'/s) from the group's reciprocal, hardware RNE conversions; q - z is an
                // integer |.| <= 510, exact in fp16, so only the product is rounded
                const float sh = (float)(_Float16)cs;
#if AWQ_ACT_MIX_DQ
                h2v dqp[EPL / 2];     // (q - z) * sh rounded to fp16, two per register
                if constexpr (DT != AWQ_DTYPE_F32 && AWQ_ACT_F16_TAIL) {
                    // bf16 / fp16 u: rint + clamp + (q - z) * s in packed fp16, as the clip search's
                    // chunk_err_bf16h (u exact in fp16 where it matters; oracle/verify_recip.c
                    // chain16): RN_f16(u + 1024 - qmin) clamped to [1024, 1024 + qmax - qmin], minus
                    // 1024 - qmin + z (exact), times the fp16 scale (one rounding of the exact product)
                    const _Float16 off = (_Float16)(1024 - qmin), hi1 = (_Float16)(1024 + qmax - qmin);
                    const _Float16 qz1 = off + (_Float16)cz, sh1 = (_Float16)sh;
                    const h2v offv = {off, off}, lov = {(_Float16)1024, (_Float16)1024}, hiv = {hi1, hi1};
                    const h2v qzv = {qz1, qz1}, shv = {sh1, sh1};
                    if constexpr (kF16Packed) {
                        // fp16: t from the packed w' directly (v_fma_mix_f32 reads the fp16 halves),
                        // RN_f16 two at a time, + z as v_pk_add_f16 (RN_f16 of the exact sum: f32's
                        // 24 bits >= 2 * 11 + 2 make torch's f32-then-fp16 rounding the same)
                        const _Float16 czh = (_Float16)cz;
                        const h2v czv = {czh, czh};
                        auto tail16 = [&](auto plain) {
#pragma unroll
                            for (int k = 0; k < EPL / 2; ++k) {
                                float p0, p1;
                                if constexpr (decltype(plain)::value) {
                                    p0 = mprod_h<false>(wsp[k], r);
                                    p1 = mprod_h<true>(wsp[k], r);
                                } else {
                                    p0 = mquot_h<false>(wsp[k], cs, r);
                                    p1 = mquot_h<true>(wsp[k], cs, r);
                                }
                                const h2v th = __builtin_convertvector((f2){opq(p0), opq(p1)}, h2v);
                                const h2v uh = sym ? th : th + czv;
                                const h2v q = __builtin_elementwise_min(__builtin_elementwise_max(uh + offv, lov), hiv);
                                dqp[k] = (q - qzv) * shv;
                            }
                        };
                        if (AWQ_ACT_F16_PLAIN && __builtin_amdgcn_ballot_w64(!(cs < 14.0f)) == 0)
                            tail16(std::true_type{});
                        else
                            tail16(std::false_type{});
                    } else {
                    auto tail = [&](auto plain) {
#pragma unroll
                        for (int j = 0; j < EPL; j += 2) {
                            float uu[2];
                            if constexpr (DT == AWQ_DTYPE_BF16 && AWQ_ACT_PK_F32) {
                                // bf16: RN(w' r) and RN(t + z) as packed pairs (v_pk_mul_f32 /
                                // v_pk_add_f32, each half the IEEE op)
                                const f2 p = (f2){ws[j], ws[j + 1]} * (f2){r, r};
                                const float t0 = H::rn(p.x), t1 = H::rn(p.y);
                                const f2 a = (f2){t0, t1} + (f2){cz, cz};
                                uu[0] = sym ? t0 : H::rn(a.x);
                                uu[1] = sym ? t1 : H::rn(a.y);
                            } else {
#pragma unroll
                                for (int u2 = 0; u2 < 2; ++u2) {
                                    // fp16, every group of the wave with s < 14: the plain quotient
                                    // RN_f16(RN_f32(w' r)) (oracle/verify_recip.c f16s)
                                    const float t = decltype(plain)::value ? hw_rn_f16(opq(ws[j + u2] * r))
                                                                           : H::quot(ws[j + u2], cs, r);
                                    uu[u2] = sym ? t : H::rn(t + cz);
                                }
                            }
                            const h2v uh = __builtin_convertvector((float __attribute__((ext_vector_type(2)))){uu[0], uu[1]}, h2v);
                            const h2v q = __builtin_elementwise_min(__builtin_elementwise_max(uh + offv, lov), hiv);
                            dqp[j / 2] = (q - qzv) * shv;
                        }
                    };
                    if (DT == AWQ_DTYPE_F16 && AWQ_ACT_F16_PLAIN && __builtin_amdgcn_ballot_w64(!(cs < 14.0f)) == 0)
                        tail(std::true_type{});
                    else
                        tail(std::false_type{});
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < EPL; j += 2) {
                        float qq[2];
#pragma unroll
                        for (int u2 = 0; u2 < 2; ++u2) {
                            const float t = H::quot(ws[j + u2], cs, r);
                            const float u = sym ? t : H::rn(t + cz);
                            qq[u2] = __builtin_amdgcn_fmed3f(__builtin_rintf(u), (float)qmin, (float)qmax);
                        }
                        dqp[j / 2] = (h2v){(_Float16)opq((qq[0] - cz) * sh), (_Float16)opq((qq[1] - cz) * sh)};
                    }
                }
                auto dqf = [&](int j) { return (float)dqp[j / 2][j & 1]; };
#else
                float dq[EPL];
#pragma unroll
                for (int j = 0; j < EPL; ++j) {
                    const float t = H::quot(ws[j], cs, r);
                    const float u = sym ? t : H::rn(t + cz);
                    const float q = __builtin_amdgcn_fmed3f(__builtin_rintf(u), (float)qmin, (float)qmax);
                    dq[j] = hw_rn_f16((q - cz) * sh);
                }
                auto dqf = [&](int j) { return dq[j]; };
#endif
                auto ieee = [&]() {
#pragma unroll
                    for (int c = 0; c < EPL / 8; ++c) acc[c] = 0.0f;
#pragma unroll
                    for (int j = 0; j < EPL; ++j) {
                        const float e = dqf(j) / s[j] - v[j];
                        acc[j / 8] = acc[j / 8] + h[j] * (e * e);
                    }
                };
                if (mq) {
#pragma unroll
                    for (int j = 0; j < EPL; ++j) {
#if AWQ_ACT_MIX_DQ
                        const float w_hat = (j & 1) ? mquot_h<true>(dqp[j / 2], s[j], rs[j])
                                                    : mquot_h<false>(dqp[j / 2], s[j], rs[j]);
#else
                        const float w_hat = mquot(dqf(j), s[j], rs[j]);
#endif
                        const float e = w_hat - v[j];
                        acc[j / 8] = acc[j / 8] + h[j] * (e * e);
                    }
#if AWQ_ACT_NAN_RTABLE
                    // a NaN loss: an out-of-range reciprocal (NaN), or a NaN / inf statistic —
                    // the wave redoes the candidate with IEEE divisions (same bits in range)
                    bool bad = false;
#pragma unroll
                    for (int c = 0; c < EPL / 8; ++c) bad |= acc[c] != acc[c];
                    if (__builtin_expect(__builtin_amdgcn_ballot_w64(bad) != 0, 0)) ieee();
#endif
                } else {
                    ieee();
                }
            } else {
                const float sh = sw_f16_to_f32(canon_f16(cs));
#pragma unroll
                for (int j = 0; j < EPL; ++j) {
                    const float q = quant1<DT>(ws[j], cs, cz, qmin, qmax);
                    const float hq = sw_f16_to_f32(sw_f32_to_f16(q - cz));
                    const float dq = sw_f16_to_f32(sw_f32_to_f16(hq * sh));
                    const float e = dq / s[j] - v[j];
                    acc[j / 8] = acc[j / 8] + h[j] * (e * e);
                }
            }
            float a = acc[0];
            if (EPL == 16) a = acc[0] + acc[EPL / 8 - 1];
            a = grp_sum(a, lpg);
            if constexpr (kLds) {
                // one store that every lane issues (no branch around it: the wait before the
                // next candidate's LDS reads can then leave this store in flight); lanes other
                // than valid group leaders address past the buffer range and write nothing
                const uint32_t off = (gl.valid && leader) ? (uint32_t)((gl.r * G + gl.g) * 4) : 0x80000000u;
                __builtin_amdgcn_raw_buffer_store_b32(
                    __float_as_uint(a), act_rsrc(part + (int64_t)i * stride, (uint32_t)(stride * 4)), off, 0, 0);
            } else if (gl.valid && leader) {
                part[(int64_t)i * stride + gl.r * G + gl.g] = a;
            }
        }
    }
}

// work[i * nblk + b] = block b of candidate i's losses, fp64: 64-group sub-blocks summed
// ascending, then the block's 16 sub-block sums ascending.  A workgroup takes kLossChains
// consecutive (i, b) blocks: their floats come in through LDS with coalesced loads (all in
// flight at once), every thread runs one sub-block chain from LDS, kLossChains lanes add the
// sub-block sums.  LDS layout: block c's sub-block u at c * 1024 + 64 u, its 64 floats
// rotated by (u + 16 c) mod 64 so that the 64 lanes of a wave (4 blocks x 16 sub-blocks)
// read 64 distinct banks at every step of their chains.
constexpr int kLossChains = 16;   // r92: 8 or 4 blocks per workgroup were 5-30 % slower
constexpr int kLossSubs = kGroupBlock / kGroupSub;
static_assert(kLossChains * kLossSubs == 256, "one sub-block chain per thread");
__device__ __forceinline__ int loss_lds_index(int c, int g) {
    return c * kGroupBlock + (g & ~(kGroupSub - 1)) + ((g + (g >> 6) + 16 * c) & (kGroupSub - 1));
}
__global__ __launch_bounds__(256) void loss_block_kernel(const float* __restrict__ part, int n_grid, int64_t stride,
                                                         int64_t nblk, double* __restrict__ work) {
    __shared__ __attribute__((aligned(16))) float sp[kLossChains * kGroupBlock];
    __shared__ double su[kLossChains][kLossSubs];
    const int tid = threadIdx.x;
    const int64_t c0 = (int64_t)blockIdx.x * kLossChains;
    const int64_t nch = (int64_t)n_grid * nblk;
    // every load first (64 per thread in flight), then the LDS stores: a load -> store loop
    // would wait out one memory round trip per element
    constexpr int NE = kGroupBlock / 256;
    float t[kLossChains][NE];
#pragma unroll
    for (int c = 0; c < kLossChains; ++c) {
        const int64_t idx = (c0 + c < nch) ? c0 + c : nch - 1;
        const int64_t i = idx / nblk, b = idx - i * nblk;
        const int64_t g0 = b * kGroupBlock;
        const int64_t n = (g0 + kGroupBlock < stride) ? kGroupBlock : stride - g0;
        const float* p = part + i * stride + g0;
#pragma unroll
        for (int e = 0; e < NE; ++e) t[c][e] = (e * 256 + tid < n) ? p[e * 256 + tid] : 0.0f;
    }
#pragma unroll
    for (int c = 0; c < kLossChains; ++c)
#pragma unroll
        for (int e = 0; e < NE; ++e) sp[loss_lds_index(c, e * 256 + tid)] = t[c][e];
    __syncthreads();
    {
        const int c = tid / kLossSubs, u = tid % kLossSubs;
        const int64_t idx = c0 + c;
        int n = 0;
        if (idx < nch) {
            const int64_t b = idx % nblk, g0 = b * kGroupBlock;
            n = (int)((g0 + kGroupBlock < stride) ? kGroupBlock : stride - g0);
        }
        const int ga = u * kGroupSub, gb = min(ga + kGroupSub, n);
        const float* q = sp + c * kGroupBlock + ga;
        const int rot = (ga / kGroupSub + 16 * c) & (kGroupSub - 1);   // (g >> 6) == u here
        double s = 0.0;
        for (int g = ga; g < gb; g += 16) {               // 16 LDS values ahead of the chain
            float v[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) v[j] = q[(g - ga + j + rot) & (kGroupSub - 1)];
#pragma unroll
            for (int j = 0; j < 16; ++j)
                if (g + j < gb) s += (double)v[j];
        }
        su[c][u] = s;
    }
    __syncthreads();
    const int64_t idx = c0 + tid;
    if (tid >= kLossChains || idx >= nch) return;
    const int64_t b = idx % nblk, g0 = b * kGroupBlock;
    const int n = (int)((g0 + kGroupBlock < stride) ? kGroupBlock : stride - g0);
    double s = 0.0;
    for (int u = 0; u < kLossSubs && u * kGroupSub < n; ++u) s += su[tid][u];   // non-empty, ascending
    work[idx] = s;
}

// losses[i] = the candidate's blocks summed in 32-block super-blocks (blocks ascending),
// then the super-block sums ascending (fp64); best = first minimum (NaN never wins; all NaN
// -> 0); s_best = table[best].  Candidates go in batches whose super-block sums fit LDS:
// every thread runs (candidate, super-block) chains of <= 32 block sums from global memory
// (loads first, then the adds), then one lane per candidate adds its super-block sums.
constexpr int kSelectLds = 6144;   // fp64 super-block sums per batch (48 KiB)
__global__ __launch_bounds__(256) void select_kernel(const double* __restrict__ work, int n_grid, int64_t nblk,
                                                     const float* __restrict__ table, int64_t K,
                                                     double* __restrict__ losses, int32_t* __restrict__ best,
                                                     float* __restrict__ s_best) {
    __shared__ double sw[kSelectLds];
    __shared__ double sl[AWQ_ACT_MAX_GRID];
    __shared__ int sb;
    const int tid = threadIdx.x;
    const int nsb = (int)((nblk + kSuperBlocks - 1) / kSuperBlocks);   // host-checked <= kSelectLds
    const int per = kSelectLds / nsb;                                  // candidates per batch
    for (int i0 = 0; i0 < n_grid; i0 += per) {
        const int nc = min(per, n_grid - i0);
        for (int it = tid; it < nc * nsb; it += 256) {
            const int ci = it / nsb, q = it - ci * nsb;
            const int64_t b0 = (int64_t)q * kSuperBlocks;
            const int nb = (int)min((int64_t)kSuperBlocks, nblk - b0);
            const double* p = work + (int64_t)(i0 + ci) * nblk + b0;
            double v[kSuperBlocks];
#pragma unroll
            for (int j = 0; j < kSuperBlocks; ++j) v[j] = p[j < nb ? j : nb - 1];
            double s = 0.0;
#pragma unroll
            for (int j = 0; j < kSuperBlocks; ++j)
                if (j < nb) s += v[j];
            sw[it] = s;
        }
        __syncthreads();
        if (tid < nc) {
            double s = 0.0;
            for (int q = 0; q < nsb; ++q) s += sw[tid * nsb + q];
            sl[i0 + tid] = s;
            if (losses) losses[i0 + tid] = s;
        }
        __syncthreads();
    }
    if (tid == 0) {
        double bv = __builtin_inf();
        int bi = 0;
        for (int i = 0; i < n_grid; ++i)
            if (sl[i] < bv) { bv = sl[i]; bi = i; }
        sb = bi;
        if (best) best[0] = bi;
    }
    __syncthreads();
    if (s_best)
        for (int64_t k = tid; k < K; k += 256) s_best[k] = table[(int64_t)sb * K + k];
}

// out = RN_D(w * s[k]) (torch: W.mul_(scales) on a D tensor with an fp32 scale vector);
// 8 consecutive elements of one row per lane (K % 8 == 0), vector loads / stores
template <int DT>
__global__ __launch_bounds__(256) void apply_scale_kernel(const void* __restrict__ w, int64_t R, int64_t K,
                                                          const float* __restrict__ s, void* __restrict__ out) {
    typedef Traits<DT> T;
    const int64_t n8 = R * K / 8;
    for (int64_t o = (int64_t)blockIdx.x * 256 + threadIdx.x; o < n8; o += (int64_t)gridDim.x * 256) {
        const int64_t i = o * 8;
        const int64_t k = i % K;
        float v[8], y[8];
        load8<DT>(w, i, v);
        const float4 sa = *(const float4*)(s + k), sb = *(const float4*)(s + k + 4);
        const float sv[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = T::rn(v[j] * sv[j]);
        if (DT == AWQ_DTYPE_F32) {
            float4* q = (float4*)((float*)out + i);
            q[0] = make_float4(y[0], y[1], y[2], y[3]);
            q[1] = make_float4(y[4], y[5], y[6], y[7]);
        } else {
            uint32_t h[8];
#pragma unroll
            for (int j = 0; j < 8; ++j)
                h[j] = (DT == AWQ_DTYPE_BF16) ? (__float_as_uint(y[j]) >> 16) : (uint32_t)sw_f32_to_f16(y[j]);
            *(uint4*)((uint16_t*)out + i) = make_uint4(h[0] | (h[1] << 16), h[2] | (h[3] << 16), h[4] | (h[5] << 16),
                                                       h[6] | (h[7] << 16));
        }
    }
}

// any shape / alignment: one element per lane
template <int DT>
__global__ __launch_bounds__(256) void apply_scale_any_kernel(const void* __restrict__ w, int64_t R, int64_t K,
                                                              const float* __restrict__ s, void* __restrict__ out) {
    typedef Traits<DT> T;
    const typename T::S* p = (const typename T::S*)w;
    const int64_t total = R * K;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const float y = T::rn(T::load(p, i) * s[i % K]);
        if (DT == AWQ_DTYPE_BF16) ((uint16_t*)out)[i] = (uint16_t)(__float_as_uint(y) >> 16);
        else if (DT == AWQ_DTYPE_F16) ((uint16_t*)out)[i] = sw_f32_to_f16(y);
        else ((float*)out)[i] = y;
    }
}

inline unsigned blocks_for(int64_t work, int64_t per_block, int64_t cap) {
    int64_t b = (work + per_block - 1) / per_block;
    if (b < 1) b = 1;
    if (b > cap) b = cap;
    return (unsigned)b;
}

}  // namespace

#define AWQ_DT_SWITCH(dtype, KERNEL_CALL)                            \
    switch (dtype) {                                                 \
    case AWQ_DTYPE_BF16: { constexpr int D = AWQ_DTYPE_BF16; KERNEL_CALL; } break; \
    case AWQ_DTYPE_F16: { constexpr int D = AWQ_DTYPE_F16; KERNEL_CALL; } break;   \
    case AWQ_DTYPE_F32: { constexpr int D = AWQ_DTYPE_F32; KERNEL_CALL; } break;   \
    default: return hipErrorInvalidValue;                            \
    }

hipError_t launch_act_stats(const void* x, int dtype, int64_t T, int64_t K, double* work, float* x_mean,
                            float* x_sq, hipStream_t stream) {
    const int64_t nblk = (T + kRowBlock - 1) / kRowBlock;
    double* p0 = work;
    double* p1 = work + nblk * K;
    if (K % 8 == 0 && (uintptr_t)x % 16 == 0) {
        const dim3 gt((unsigned)((K + kColTile - 1) / kColTile), (unsigned)nblk);
        AWQ_DT_SWITCH(dtype, hipLaunchKernelGGL((colsum_tile_kernel<D, 0>), gt, dim3(256), 0, stream, x, T, K, K,
                                                nullptr, p0, p1))
    } else {
        const dim3 grid((unsigned)((K + 255) / 256), (unsigned)nblk);
        AWQ_DT_SWITCH(dtype, hipLaunchKernelGGL((colsum_kernel<D, 0>), grid, dim3(256), 0, stream, x, T, K, K,
                                                nullptr, p0, p1))
    }
    if (hipError_t e = hipPeekAtLastError()) return e;
    const dim3 g1((unsigned)((K + 255) / 256));
    hipLaunchKernelGGL(colmean_kernel, g1, dim3(256), 0, stream, p0, nblk, K, (double)T, x_mean);
    hipLaunchKernelGGL(colmean_kernel, g1, dim3(256), 0, stream, p1, nblk, K, (double)T, x_sq);
    return hipPeekAtLastError();
}

hipError_t launch_weight_colsum(const void* w, int dtype, int64_t R, int64_t K, int64_t L, float* gmax,
                                double* part, hipStream_t stream) {
    const int64_t nb = (R + kRowBlock - 1) / kRowBlock;
    if (AWQ_WMEAN_FUSED && (L == 32 || L == 64 || L == 128 || L == 256) && K % L == 0 && (uintptr_t)w % 16 == 0) {
        const dim3 gf((unsigned)(K / L), (unsigned)nb);
#define AWQ_WCF(G) AWQ_DT_SWITCH(dtype, hipLaunchKernelGGL((wcolsum_fused_kernel<D, G>), gf, dim3(256), 0, stream, w, R, K, part))
        switch (L) {
        case 32: AWQ_WCF(32) break;
        case 64: AWQ_WCF(64) break;
        case 128: AWQ_WCF(128) break;
        default: AWQ_WCF(256) break;
        }
#undef AWQ_WCF
        return hipPeekAtLastError();
    }
    const int lpg = (int)(L / 8);
    const int64_t G = K / L;
    const int64_t items = ((R + (64 / lpg) - 1) / (64 / lpg)) * G;
    AWQ_DT_SWITCH(dtype, hipLaunchKernelGGL((group_absmax_kernel<D>), dim3(blocks_for(items, 4, 256 * 64)),
                                            dim3(256), 0, stream, w, R, K, lpg, gmax))
    if (hipError_t e = hipPeekAtLastError()) return e;
    const int64_t nblk = (R + kRowBlock - 1) / kRowBlock;
    if (K % 8 == 0 && L % 8 == 0 && (uintptr_t)w % 16 == 0) {
        const dim3 gt((unsigned)((K + kColTile - 1) / kColTile), (unsigned)nblk);
        AWQ_DT_SWITCH(dtype, hipLaunchKernelGGL((colsum_tile_kernel<D, 1>), gt, dim3(256), 0, stream, w, R, K, L,
                                                gmax, part, nullptr))
    } else {
        const dim3 grid((unsigned)((K + 255) / 256), (unsigned)nblk);
        AWQ_DT_SWITCH(dtype, hipLaunchKernelGGL((colsum_kernel<D, 1>), grid, dim3(256), 0, stream, w, R, K, L, gmax,
                                                part, nullptr))
    }
    return hipPeekAtLastError();
}

hipError_t launch_colmean(const double* part, int64_t nblk, int64_t K, double divisor, float* out,
                          hipStream_t stream) {
    hipLaunchKernelGGL(colmean_kernel, dim3((unsigned)((K + 255) / 256)), dim3(256), 0, stream, part, nblk, K,
                       divisor, out);
    return hipPeekAtLastError();
}

hipError_t launch_scale_table_ws(const float* x_mean, const float* w_mean, int64_t K, int n_grid, double* work,
                                 float* table, hipStream_t stream) {
    const int64_t S = (K + kTabSlice - 1) / kTabSlice;
    double* raw = work;
    double* part = work + (int64_t)n_grid * K;
    const dim3 grid((unsigned)S, (unsigned)n_grid);
    hipLaunchKernelGGL(table_raw_kernel, grid, dim3(kTabSlice), 0, stream, x_mean, w_mean, K, n_grid, raw, part);
    if (hipError_t e = hipPeekAtLastError()) return e;
    hipLaunchKernelGGL(table_norm_kernel, grid, dim3(kTabSlice), 0, stream, raw, part, K, table);
    return hipPeekAtLastError();
}

hipError_t launch_scale_table(const float* x_mean, const float* w_mean, int64_t K, int n_grid, float* table,
                              hipStream_t stream) {
    // the normalising max / min pass is repeated by each slice's workgroup (no cross-workgroup
    // exchange); the second pow pass is split over the slices
    const unsigned slices = (unsigned)((K + 2 * kTableThreads - 1) / (2 * kTableThreads) < 8
                                           ? (K + 2 * kTableThreads - 1) / (2 * kTableThreads) : 8);
    hipLaunchKernelGGL(scale_table_kernel, dim3((unsigned)n_grid, slices), dim3(kTableThreads), 0, stream, x_mean,
                       w_mean, K, n_grid, table);
    return hipPeekAtLastError();
}

// rtable[i] = RN_f32(1 / table[i]) inside [2^-60, 2^60] (mquot's proven range), else a NaN
// (AWQ_ACT_NAN_RTABLE: a quotient through it is NaN, which sends its wave to the IEEE division;
// 0 in the round-5 encoding, checked per wave and candidate)
__global__ __launch_bounds__(256) void recip_table_kernel(const float* __restrict__ table, int64_t n,
                                                          float* __restrict__ rtable) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float s = table[i];
    rtable[i] = (s >= 0x1p-60f && s <= 0x1p60f) ? 1.0f / s : (AWQ_ACT_NAN_RTABLE ? __builtin_nanf("") : 0.0f);
}

// awq_selftest 1: mquot == IEEE division for every s in [1, 2) (all 2^23 mantissas) and every
// positive finite fp16 a; counts mismatches
__global__ __launch_bounds__(256) void selftest_mquot_kernel(unsigned long long* mismatches) {
    const uint32_t m = blockIdx.x * 256 + threadIdx.x;
    if (m >= (1u << 23)) return;
    const float s = __uint_as_float(0x3F800000u | m);
    const float rs = 1.0f / s;
    unsigned long long bad = 0;
    for (uint32_t h = 1; h < 0x7C00u; ++h) {
        const float a = (float)__builtin_bit_cast(_Float16, (uint16_t)h);
        bad += __float_as_uint(mquot(a, s, rs)) != __float_as_uint(a / s);
    }
    if (bad) atomicAdd(mismatches, bad);
}

hipError_t launch_recip_table(const float* table, int64_t n, float* rtable, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(recip_table_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, table, n, rtable);
    return hipPeekAtLastError();
}

hipError_t launch_selftest_mquot(unsigned long long* out, hipStream_t stream) {
    hipLaunchKernelGGL(selftest_mquot_kernel, dim3((1u << 23) / 256), dim3(256), 0, stream, out);
    return hipPeekAtLastError();
}

hipError_t launch_act_losses(const void* w, int dtype, int64_t R, int64_t K, int64_t L, int bits, int symmetric,
                             const float* table, const float* rtable, int n_grid, const float* x_sq, float* part,
                             int64_t stride, hipStream_t stream) {
    const int qmin = symmetric ? -(1 << (bits - 1)) : 0;
    const int qmax = symmetric ? (1 << (bits - 1)) - 1 : (1 << bits) - 1;
    const int lpg = (int)(L / 8);
    const int64_t items = ((R + (64 / lpg) - 1) / (64 / lpg)) * (K / L);
    const unsigned grid = blocks_for(items, 4, 256 * 32);
#define AWQ_LOSS_LAUNCH(LP, SY, EP, LPA)                                                                       \
    AWQ_DT_SWITCH(dtype, hipLaunchKernelGGL((act_loss_kernel<D, LP, SY, EP>), dim3(g2), dim3(256), 0, stream, w, R, \
                                            K, LPA, qmin, qmax, table, rtable, n_grid, x_sq, part, stride))
#define AWQ_LOSS_SYM(LP, EP, LPA)                                                   \
    if (symmetric) { AWQ_LOSS_LAUNCH(LP, true, EP, LPA) } else { AWQ_LOSS_LAUNCH(LP, false, EP, LPA) }
    // the streaming group sizes 32 / 64 / 128 / 256: 16 elements per lane, gs / 16 lanes per
    // group as a constant (twice the groups per wave: half the items)
    const unsigned g2 = (lpg >= 4 && lpg <= 32) ? blocks_for((items + 1) / 2, 4, 256 * 32) : grid;
    switch (lpg) {
    case 4: AWQ_LOSS_SYM(2, 16, 2) break;
    case 8: AWQ_LOSS_SYM(4, 16, 4) break;
    case 16: AWQ_LOSS_SYM(8, 16, 8) break;
    case 32: AWQ_LOSS_SYM(16, 16, 16) break;
    default: AWQ_LOSS_SYM(0, 8, lpg) break;
    }
#undef AWQ_LOSS_SYM
#undef AWQ_LOSS_LAUNCH
    return hipPeekAtLastError();
}

hipError_t launch_act_select(const float* part, int n_grid, int64_t stride, const float* table, int64_t K,
                             double* work, double* losses, int32_t* best, float* s_best, hipStream_t stream) {
    const int64_t nblk = (stride + kGroupBlock - 1) / kGroupBlock;
    if (n_grid < 1 || n_grid > AWQ_ACT_MAX_GRID || (nblk + kSuperBlocks - 1) / kSuperBlocks > kSelectLds)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(loss_block_kernel, dim3(blocks_for((int64_t)n_grid * nblk, kLossChains, INT32_MAX)), dim3(256),
                       0, stream, part, n_grid, stride, nblk, work);
    if (hipError_t e = hipPeekAtLastError()) return e;
    hipLaunchKernelGGL(select_kernel, dim3(1), dim3(256), 0, stream, work, n_grid, nblk, table, K, losses, best,
                       s_best);
    return hipPeekAtLastError();
}

hipError_t launch_apply_scale(const void* w, int dtype, int64_t R, int64_t K, const float* s, void* out,
                              hipStream_t stream) {
    const bool vec = K % 8 == 0 && ((uintptr_t)w | (uintptr_t)s | (uintptr_t)out) % 16 == 0;
    if (!vec) {
        const unsigned g1 = blocks_for(R * K, 256, 256 * 64);
        AWQ_DT_SWITCH(dtype, hipLaunchKernelGGL((apply_scale_any_kernel<D>), dim3(g1), dim3(256), 0, stream, w, R, K,
                                                s, out))
        return hipPeekAtLastError();
    }
    const unsigned grid = blocks_for(R * K / 8, 256, 256 * 64);
    AWQ_DT_SWITCH(dtype, hipLaunchKernelGGL((apply_scale_kernel<D>), dim3(grid), dim3(256), 0, stream, w, R, K, s,
                                            out))
    return hipPeekAtLastError();
}

#undef AWQ_DT_SWITCH

}  // namespace awq
