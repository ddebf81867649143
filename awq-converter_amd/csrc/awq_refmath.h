// awq_refmath.h — device-side restatement of the reference's per-op arithmetic (torch CPU
// semantics: fp32 math, fp64 for fp64 inputs, round-to-nearest-even to the input dtype
// after every op; software conversions independent of the hardware ones), shared by the
// generic kernel (awq_generic.hip) and the activation-aware search (awq_actsearch.hip).
#pragma once

#include "awq_internal.h"

namespace awq {
namespace refmath {

// ---- software RNE conversions (bit-exact with c10::BFloat16 / c10::Half) ----
__device__ __forceinline__ float sw_rn_bf16(float f) {
    if (__builtin_isnan(f)) return f;
    uint32_t u = __float_as_uint(f);
    u += 0x7FFFu + ((u >> 16) & 1u);
    return __uint_as_float(u & 0xFFFF0000u);
}

__device__ __forceinline__ uint16_t sw_f32_to_f16(float f) {
    uint32_t x = __float_as_uint(f);
    uint16_t sign = (uint16_t)((x >> 16) & 0x8000u);
    uint32_t ax = x & 0x7FFFFFFFu;
    if (ax > 0x7F800000u) return (uint16_t)(sign | 0x7E00u | ((ax >> 13) & 0x3FFu));
    if (ax >= 0x47800000u) return (uint16_t)(sign | 0x7C00u);
    if (ax >= 0x38800000u) {
        uint32_t e = (ax >> 23) - 127u + 15u;
        uint32_t m = ax & 0x7FFFFFu;
        uint32_t h = (e << 10) | (m >> 13);
        uint32_t rem = m & 0x1FFFu;
        if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
        return (uint16_t)(sign | h);
    }
    float m = __builtin_rintf(__uint_as_float(ax) * 16777216.0f);
    return (uint16_t)(sign | (uint16_t)m);
}

__device__ __forceinline__ float sw_f16_to_f32(uint16_t h) {
    uint32_t sign = ((uint32_t)h & 0x8000u) << 16;
    uint32_t e = (h >> 10) & 0x1Fu, m = h & 0x3FFu;
    if (e == 0x1F) return __uint_as_float(sign | 0x7F800000u | (m << 13));
    if (e == 0) {
        float v = (float)m * (1.0f / 16777216.0f);
        return sign ? -v : v;
    }
    return __uint_as_float(sign | ((e - 15u + 127u) << 23) | (m << 13));
}

__device__ __forceinline__ uint16_t canon_f16(float s) {
    return __builtin_isnan(s) ? (uint16_t)0x7E00 : sw_f32_to_f16(s);
}

// ---- dtype traits: storage type, compute type, per-op rounding ----
template <int DT> struct Traits;
template <> struct Traits<AWQ_DTYPE_BF16> {
    typedef uint16_t S; typedef float C;
    static __device__ float load(const S* p, int64_t i) { return __uint_as_float((uint32_t)p[i] << 16); }
    static __device__ float rn(float v) { return sw_rn_bf16(v); }
    static __device__ float lo() { return __uint_as_float(0x2EDC0000u); }   // RN_bf16(1e-10)
    static __device__ S store(float v) { return (S)(__float_as_uint(sw_rn_bf16(v)) >> 16); }
};
template <> struct Traits<AWQ_DTYPE_F16> {
    typedef uint16_t S; typedef float C;
    static __device__ float load(const S* p, int64_t i) { return sw_f16_to_f32(p[i]); }
    static __device__ float rn(float v) { return sw_f16_to_f32(sw_f32_to_f16(v)); }
    static __device__ float lo() { return 0.0f; }                           // RN_f16(1e-10) = 0
    static __device__ S store(float v) { return sw_f32_to_f16(v); }
};
template <> struct Traits<AWQ_DTYPE_F32> {
    typedef float S; typedef float C;
    static __device__ float load(const S* p, int64_t i) { return p[i]; }
    static __device__ float rn(float v) { return v; }
    static __device__ float lo() { return 1e-10f; }
    static __device__ S store(float v) { return v; }
};
template <> struct Traits<AWQ_DTYPE_F64> {
    typedef double S; typedef double C;
    static __device__ double load(const S* p, int64_t i) { return p[i]; }
    static __device__ double rn(double v) { return v; }
    static __device__ double lo() { return 1e-10; }
    static __device__ S store(double v) { return v; }
};

template <typename C> __device__ __forceinline__ C wave_min(C v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { C t = __shfl_xor(v, o, 64); v = t < v ? t : v; }
    return v;
}
template <typename C> __device__ __forceinline__ C wave_max(C v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { C t = __shfl_xor(v, o, 64); v = t > v ? t : v; }
    return v;
}
__device__ __forceinline__ int wave_or(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ float absv(float v) { return __builtin_fabsf(v); }
__device__ __forceinline__ double absv(double v) { return __builtin_fabs(v); }
__device__ __forceinline__ float rnd(float v) { return __builtin_rintf(v); }
__device__ __forceinline__ double rnd(double v) { return __builtin_rint(v); }

template <typename C> __device__ __forceinline__ C clampq(C v, C lo, C hi) {   // NaN propagates
    if (v != v) return v;
    return v < lo ? lo : (v > hi ? hi : v);
}
template <typename C> __device__ __forceinline__ int32_t to_i32(C v) {         // NaN -> INT_MIN
    return (v != v) ? INT32_MIN : (int32_t)v;
}

template <typename C> __device__ __forceinline__ C wave_sum(C v) {
    // xor butterfly with growing offsets = the pairwise tree over adjacent lanes: lanes l
    // and l^o add the same two values, so every lane ends with the same sum
    // (oracle_quantize_search restates this tree; the streaming kernel's 16-lane DPP
    // reduction is the same tree's first four levels)
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v = v + __shfl_xor(v, o, 64);
    return v;
}

// awq.py:196-213: scale and zero point of one group from its (NaN-propagated) min/max.
// torch_gpu: as torch's GPU kernels evaluate the same lines (a reference quantizer with
// device="cuda"): the division by the Python int qmax - qmin is a product with the opmath
// reciprocal RN(1 / (qmax - qmin)) (ATen's div_true_kernel_cuda for a CPU-scalar divisor), and
// clamp(-0, 0, qmax) is +0 (the GPU clamp's IEEE maximum).
template <int DT>
__device__ __forceinline__ void group_params(typename Traits<DT>::C mn, typename Traits<DT>::C mx, int nan,
                                             int qmin, int qmax, int sym, typename Traits<DT>::C& s_out,
                                             typename Traits<DT>::C& z_out, bool torch_gpu = false) {
    typedef Traits<DT> T;
    typedef typename T::C C;
    if (sym) {                                   // awq.py:196-199 (Python max)
        C amn = absv(mn), amx = absv(mx);   // torch.abs(-0) = +0
        if (nan) { amn = mn; amx = mx; }
        C a = (amx > amn) ? amx : amn;
        mn = -a;
        mx = a;
    }
    C s = torch_gpu ? T::rn(T::rn(mx - mn) * ((C)1 / (C)(qmax - qmin)))   // awq.py:202
                    : T::rn(T::rn(mx - mn) / (C)(qmax - qmin));
    if (!(s != s) && s < T::lo()) s = T::lo();                 // awq.py:205
    C z = (C)0;
    if (!sym) {                                                // awq.py:210-211
        C y = T::rn(mn / s);
        z = T::rn((C)qmin - y);
        z = clampq(T::rn(rnd(z)), (C)qmin, (C)qmax);
        if (torch_gpu && z == (C)0) z = (C)0;                  // GPU clamp: max(-0, +0) = +0
    }
    s_out = s;
    z_out = z;
}

template <int DT>
__device__ __forceinline__ typename Traits<DT>::C quant1(typename Traits<DT>::C v, typename Traits<DT>::C s,
                                                         typename Traits<DT>::C z, int qmin, int qmax) {
    typedef Traits<DT> T;
    typedef typename T::C C;
    C t = T::rn(T::rn(v / s) + z);                     // awq.py:245
    return clampq(T::rn(rnd(t)), (C)qmin, (C)qmax);    // awq.py:248
}

}  // namespace refmath
}  // namespace awq
