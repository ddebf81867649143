// awq_generic.hip — any-dtype / any-group-size quantizer, packer and dequantizer (gfx950).
//
// Covers every case the streaming kernel (awq_fast.hip) does not: fp16/fp32/fp64 inputs,
// group sizes other than 128, K not a multiple of the group size (zero-padded tail group,
// reference awq.py:337-339) and the small-tensor path (numel < group_size, awq.py:130-171,
// expressed by the caller as one group per row: group_size = K).
//
// One wave per span of groups (one qzeros word): lanes stride over a group's elements,
// min/max/NaN reduced across the wave with cross-lane shuffles, then a pass over the span
// (L1/L2-hot) quantizes and packs.  Each
// element-wise op of the reference is evaluated the way torch's CPU kernels do for the
// input dtype D: fp32 math (fp64 for D = fp64), then round-to-nearest-even to D
// (software RNE here — independent of the hardware conversions the fast kernel uses),
// and a true IEEE division for x / s.
#include "awq_refmath.h"

#include <cstdlib>

namespace awq {
namespace {

using namespace refmath;

// SEARCH (opt-in scale_method="search"; no reference counterpart): before
// the RTN parameters are taken, the group's [min, max] is shrunk by alpha_i = (n_grid-i)/n_grid,
// i < n_cand, and the candidate whose dequantized group (the reference's dequantize:
// fp16(fp16(q - z) * fp16(s)), awq.py:459-539) has the smallest squared error wins; ties and
// NaN/inf groups keep i = 0, i.e. exactly the RTN result.  Group size <= 512 (one 8-element
// chunk per lane).
//
// One wave per SPAN = the PER = 32 / bits consecutive groups of a row whose zero points share
// one qzeros word (the row's last span may hold fewer).  A span starts at element s * PER * L
// of its row, a multiple of PER, so its packed qweight words are whole too: after the
// per-group passes (min/max/NaN, then the parameters), one pass over the span quantizes lane
// by lane (element span0 + 64 i + lane, its group found by a running index) and ORs each
// aligned run of PER lanes into one qweight word with cross-lane shuffles.  qweight / qzeros
// are written directly for every group size (no int32 staging, no pack pass: round 1 staged
// 4 B per element and re-read it); tensor_q / zeros / scales / exact parameters are optional.
// fp16 bits of a group's scale (awq.py:411; fp64 via the fp32 buffer of awq.py:327).  NaN
// scales per nan_scale_code / nan_scale_one (awq_internal.h): a one-element group (L = 1)
// keeps its element's NaN, larger groups take the dtype's pattern.
template <int DT>
__device__ __forceinline__ uint16_t gen_scale_bits(typename Traits<DT>::C s, int nan, int64_t L, int sym, int small,
                                                   const typename Traits<DT>::S* w, int64_t at) {
    if (!(s != s)) return sw_f32_to_f16((float)s);
    if (L == 1) {
        uint64_t e;
        if constexpr (DT == AWQ_DTYPE_F64) e = (uint64_t)__double_as_longlong(w[at]);
        else if constexpr (DT == AWQ_DTYPE_F32) e = __float_as_uint(w[at]);
        else e = w[at];
        return nan_scale_one(DT, sym, small != 0, e, nan != 0);
    }
    return nan_scale_pick(nan_scale_code(DT, sym, small != 0), nan != 0);
}

template <int DT, bool SEARCH>
__global__ __launch_bounds__(256) void awq_generic_kernel(const void* __restrict__ wv, int64_t rows,
                                                          int64_t K, int64_t L, int bits, int qmin, int qmax,
                                                          int sym, int small, int n_grid, int n_cand,
                                                          int32_t* __restrict__ tensor_q,
                                                          uint16_t* __restrict__ scales,
                                                          int32_t* __restrict__ zeros,
                                                          int32_t* __restrict__ qweight,
                                                          int32_t* __restrict__ qzeros,
                                                          double* __restrict__ s_exact,
                                                          double* __restrict__ z_exact) {
    typedef Traits<DT> T;
    typedef typename T::C C;
    const typename T::S* w = (const typename T::S*)wv;
    const int lane = threadIdx.x & 63;
    const int per = 32 / bits;                       // 8 (4-bit) or 4 (8-bit)
    const uint32_t mask = (1u << bits) - 1u;
    const int64_t G = (K + L - 1) / L;
    const int64_t SP = (G + per - 1) / per;          // spans per row = qzeros words per row
    const int64_t wpr = (K + per - 1) / per;         // qweight words per row
    const int64_t nspans = rows * SP;
    const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * 4;
    for (int64_t si = wave; si < nspans; si += nwaves) {
        const int64_t r = si / SP, sp = si - r * SP;
        const int64_t g0 = sp * per;
        const int ng = (int)((G - g0) < per ? (G - g0) : per);
        const int64_t base = r * K;
        C sa[8], za[8];
        uint32_t zword = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            sa[j] = (C)0;
            za[j] = (C)0;
            if (j >= ng) continue;
            const int64_t gi = r * G + g0 + j;
            const int64_t k0 = (g0 + j) * L;
            int64_t k1 = k0 + L;
            const bool padded = k1 > K;                  // awq.py:337-339 zero padding
            if (k1 > K) k1 = K;
            C mn = padded ? (C)0 : (C)INFINITY, mx = padded ? (C)0 : (C)-INFINITY;
            int nan = 0;
            for (int64_t k = k0 + lane; k < k1; k += 64) {
                C v = T::load(w, base + k);
                nan |= (v != v);
                mn = v < mn ? v : mn;
                mx = v > mx ? v : mx;
            }
            mn = wave_min(mn);
            mx = wave_max(mx);
            nan = wave_or(nan);
            if (nan) { mn = (C)NAN; mx = (C)NAN; }
            if (SEARCH && !nan) {
                if (sym) {
                    C a = (absv(mx) > absv(mn)) ? absv(mx) : absv(mn);
                    mn = -a;
                    mx = a;
                }
                C best = (C)INFINITY;
                int bi = 0;
                for (int i = 0; i < n_cand; ++i) {
                    const C al = (C)(n_grid - i) / (C)n_grid;
                    C cs, cz;
                    group_params<DT>(T::rn(mn * al), T::rn(mx * al), 0, qmin, qmax, sym, cs, cz);
                    const float sh = sw_f16_to_f32(canon_f16((float)cs));
                    // canonical error sum (include/awq_hip.h): lane l sums chunk l = elements
                    // 8l .. 8l+7 of the group in order, then the pairwise tree over the lanes
                    C acc = (C)0;
                    const int64_t c0 = k0 + 8 * lane, c1 = (c0 + 8 < k1) ? c0 + 8 : k1;
                    for (int64_t k = c0; k < c1; ++k) {
                        const C v = T::load(w, base + k);
                        const C q = quant1<DT>(v, cs, cz, qmin, qmax);
                        const float h = sw_f16_to_f32(sw_f32_to_f16((float)(q - cz)));
                        const C d = v - (C)sw_f16_to_f32(sw_f32_to_f16(h * sh));
                        acc = acc + d * d;
                    }
                    acc = wave_sum(acc);
                    if (acc < best) { best = acc; bi = i; }
                }
                const C al = (C)(n_grid - bi) / (C)n_grid;
                mn = T::rn(mn * al);
                mx = T::rn(mx * al);
            }
            C s, z;
            group_params<DT>(mn, mx, nan, qmin, qmax, sym, s, z, (small & 2) != 0);
            sa[j] = s;
            za[j] = z;
            zword |= (((uint32_t)to_i32(z) - (uint32_t)qmin) & mask) << (bits * j);
            if (lane == 0) {
                if (scales) scales[gi] = gen_scale_bits<DT>(s, nan, L, sym, small & 1, w, base + k0);
                if (zeros) zeros[gi] = to_i32(z);
                if (s_exact) s_exact[gi] = (double)s;                 // the input dtype's values, exact
                if (z_exact) z_exact[gi] = (double)z;
            }
        }
        if (qzeros && lane == 0) qzeros[r * SP + sp] = (int32_t)zword;
        if (!tensor_q && !qweight) continue;
        // quantize the span: element k = span0 + 64 i + lane of group j (running index, rem = k - j L)
        const int64_t span0 = g0 * L;
        int64_t span1 = span0 + (int64_t)ng * L;
        if (span1 > K) span1 = K;
        int j = 0;
        int64_t rem = lane;
        while (rem >= L) { rem -= L; ++j; }
        const int sh = bits * (lane & (per - 1));
        for (int64_t k = span0 + lane; k - lane < span1; k += 64) {
            const bool act = k < span1;
            C s = sa[0], z = za[0];
#pragma unroll
            for (int jj = 1; jj < 8; ++jj)
                if (j == jj) { s = sa[jj]; z = za[jj]; }
            int32_t q = 0;
            if (act) q = to_i32(quant1<DT>(T::load(w, base + k), s, z, qmin, qmax));
            if (tensor_q && act) tensor_q[base + k] = q;
            if (qweight) {
                uint32_t wd = act ? (((uint32_t)q - (uint32_t)qmin) & mask) << sh : 0u;
                for (int o = 1; o < per; o <<= 1) wd |= (uint32_t)__shfl_xor((int)wd, o, 64);
                if (act && (lane & (per - 1)) == 0) qweight[r * wpr + k / per] = (int32_t)wd;
            }
            rem += 64;
            while (rem >= L) { rem -= L; ++j; }
        }
    }
}

// DPP lane moves (VALU, no LDS round trip) for the register span's in-row levels:
// quad_perm [1,0,3,2] (xor 1), quad_perm [2,3,0,1] (xor 2), row_half_mirror (lane i <-> 7 - i
// of its 8), row_mirror (i <-> 15 - i of its 16).  After xor 1 and xor 2 every lane of a quad
// holds the quad's value, so the two mirrors finish the 8- and 16-lane levels.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double x) {
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, false);
}
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppHalfMirror = 0x141, kDppMirror = 0x140;

// The same span for fp64 RTN at group sizes 64 * LPI (64, 128): the whole span (PER groups of
// LPI elements per lane) is loaded into registers with every load in flight at once, the
// per-group reductions and the quantize + pack pass run on the registers (no re-read), and a
// wave's groups are wave-uniform per register slot (slot i of every lane is in group i / LPI).
template <int LPI, int PER>
__global__ __launch_bounds__(256) void awq_generic_span_reg_kernel(const double* __restrict__ w, int64_t rows,
                                                                   int64_t K, int qmin, int qmax, int sym,
                                                                   uint32_t nan_code, int32_t* __restrict__ tensor_q,
                                                                   uint16_t* __restrict__ scales,
                                                                   int32_t* __restrict__ zeros,
                                                                   int32_t* __restrict__ qweight,
                                                                   int32_t* __restrict__ qzeros) {
    constexpr int BITS = 32 / PER, NI = LPI * PER;
    constexpr int64_t L = 64 * LPI;
    constexpr uint32_t MASK = (1u << BITS) - 1u;
    const int lane = threadIdx.x & 63;
    const int64_t G = (K + L - 1) / L;
    const int64_t SP = (G + PER - 1) / PER;
    const int64_t wpr = (K + PER - 1) / PER;
    const int64_t si = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (si >= rows * SP) return;
    const int64_t r = si / SP, sp = si - r * SP;
    const int64_t g0 = sp * PER;
    const int64_t base = r * K, span0 = g0 * L;
    double v[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {                   // zero beyond K: the reference's padding
        const int64_t k = span0 + 64 * i + lane;
        v[i] = (k < K) ? __builtin_nontemporal_load(w + base + k) : 0.0;
    }
    // lane-local min/max per group, then the PER groups' butterflies interleaved (independent
    // chains: one shuffle latency per level instead of one per level and group); NaN by ballot
    double mn[PER], mx[PER];
    uint64_t nanm[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        double a = v[j * LPI], b = a;
        int nan = a != a;
#pragma unroll
        for (int i = 1; i < LPI; ++i) {
            const double t = v[j * LPI + i];
            nan |= (t != t);
            a = t < a ? t : a;
            b = t > b ? t : b;
        }
        mn[j] = a;
        mx[j] = b;
        nanm[j] = __ballot(nan);
    }
#define AWQ_RED_LEVEL(MOVE)                                                                      \
    _Pragma("unroll") for (int j = 0; j < PER; ++j) {                                            \
        const double a = MOVE(mn[j]), b = MOVE(mx[j]);                                          \
        mn[j] = a < mn[j] ? a : mn[j];                                                           \
        mx[j] = b > mx[j] ? b : mx[j];                                                           \
    }
    AWQ_RED_LEVEL(dpp_d<kDppXor1>)
    AWQ_RED_LEVEL(dpp_d<kDppXor2>)
    AWQ_RED_LEVEL(dpp_d<kDppHalfMirror>)
    AWQ_RED_LEVEL(dpp_d<kDppMirror>)
#define AWQ_SHFL16(x) __shfl_xor((x), 16, 64)
#define AWQ_SHFL32(x) __shfl_xor((x), 32, 64)
    AWQ_RED_LEVEL(AWQ_SHFL16)
    AWQ_RED_LEVEL(AWQ_SHFL32)
#undef AWQ_SHFL16
#undef AWQ_SHFL32
#undef AWQ_RED_LEVEL
    uint32_t zword = 0;
    double sa[PER], za[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int nan = nanm[j] != 0;
        double sc, z;
        group_params<AWQ_DTYPE_F64>(nan ? NAN : mn[j], nan ? NAN : mx[j], nan, qmin, qmax, sym, sc, z);
        sa[j] = sc;
        za[j] = z;
        if (g0 + j >= G) continue;                   // wave-uniform: past the row's last group
        zword |= (((uint32_t)to_i32(z) - (uint32_t)qmin) & MASK) << (BITS * j);
        if (lane == 0) {
            const int64_t gi = r * G + g0 + j;
            if (scales) scales[gi] = sc != sc ? nan_scale_pick(nan_code, nan) : sw_f32_to_f16((float)sc);
            if (zeros) zeros[gi] = to_i32(z);
        }
    }
    if (qzeros && lane == 0) qzeros[r * SP + sp] = (int32_t)zword;
    const int sh = BITS * (lane & (PER - 1));
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int64_t k = span0 + 64 * i + lane;
        if (span0 + 64 * i >= K) break;              // wave-uniform
        const bool act = k < K;
        const int32_t q = act ? to_i32(quant1<AWQ_DTYPE_F64>(v[i], sa[i / LPI], za[i / LPI], qmin, qmax)) : 0;
        if (tensor_q && act) tensor_q[base + k] = q;
        if (qweight) {
            uint32_t wd = act ? (((uint32_t)q - (uint32_t)qmin) & MASK) << sh : 0u;
            wd |= dpp_u<kDppXor1>(wd);
            wd |= dpp_u<kDppXor2>(wd);
            if (PER == 8) wd |= dpp_u<kDppHalfMirror>(wd);
            if (act && (lane & (PER - 1)) == 0) qweight[r * wpr + k / PER] = (int32_t)wd;
        }
    }
}

// fp64 RTN for any other group size 2 <= L with the span in <= 16 KiB (4-bit: L <= 256,
// 8-bit: L <= 512): one one-wave workgroup per span (PER groups of a row), the span staged in
// LDS with every load of a batch in flight (8 per lane), then
//   pass 1  P = 64 / PER lanes per group (8 at 4-bit), each over an even share of the
//           group's elements, min / max / NaN merged over the P lanes by DPP moves (in-row);
//           the group's (s, z) by the reference arithmetic (group_params), one lane per group
//           storing scale / zero point;
//   pass 2  lane = one qweight word (PER consecutive elements): each element's group from an
//           exact float index (e + 0.5) * RN(1/L) (e < 2^13), its (s, z) from LDS, the IEEE
//           fp64 quantize (quant1), the word assembled in the lane — no cross-lane OR.
// The strided span (awq_generic_kernel) walks a wave's groups one after another with a
// 64-lane butterfly each; here every group reduces at once and the quantize pass reads LDS.
template <int PER>
__global__ __launch_bounds__(64) void awq_f64_span_lds_kernel(const double* __restrict__ w, int64_t rows, int64_t K,
                                                              int64_t L, float invL, int qmin, int qmax, int sym,
                                                              uint32_t nan_code, int32_t* __restrict__ tensor_q,
                                                              uint16_t* __restrict__ scales,
                                                              int32_t* __restrict__ zeros,
                                                              int32_t* __restrict__ qweight,
                                                              int32_t* __restrict__ qzeros) {
    constexpr int BITS = 32 / PER, P = 64 / PER;
    constexpr uint32_t MASK = (1u << BITS) - 1u;
    extern __shared__ double st[];                    // PER * L doubles
    __shared__ double sp_s[PER], sp_z[PER];
    const int lane = threadIdx.x;
    const int64_t G = (K + L - 1) / L;
    const int64_t SP = (G + PER - 1) / PER;
    const int64_t wpr = (K + PER - 1) / PER;
    const int64_t si = blockIdx.x;
    const int64_t r = si / SP, sp = si - r * SP;
    const int64_t g0 = sp * PER;
    const int64_t span0 = g0 * L;
    const int ng = (int)min((int64_t)PER, G - g0);
    const int Li = (int)L;
    const int n = (int)min((int64_t)ng * L, K - span0);   // the row's elements in the span
    const int nz = ng * Li;                                 // + the padded tail group's zeros
    const double* src = w + r * K + span0;
    for (int e0 = 0; e0 < nz; e0 += 8 * 64) {
        double v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int e = e0 + 64 * k + lane;
            v[k] = e < n ? __builtin_nontemporal_load(src + e) : 0.0;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int e = e0 + 64 * k + lane;
            if (e < nz) st[e] = v[k];
        }
    }
    __syncthreads();
    // ---- pass 1 ----
    const int grp = lane / P, j = lane % P;
    const int C = (Li + P - 1) / P;
    const int cb = min(j * C, Li), ce = min(cb + C, Li);
    double mn = INFINITY, mx = -INFINITY;
    uint32_t nan = 0;
    if (grp < ng) {
        const double* gs = st + grp * Li;
        for (int i = cb; i < ce; ++i) {
            const double t = gs[i];
            nan |= (t != t);
            mn = t < mn ? t : mn;
            mx = t > mx ? t : mx;
        }
    }
#define AWQ_F64_LEVEL(CTRL)                                   \
    {                                                         \
        const double a = dpp_d<CTRL>(mn), b = dpp_d<CTRL>(mx); \
        mn = a < mn ? a : mn;                                 \
        mx = b > mx ? b : mx;                                 \
        nan |= dpp_u<CTRL>(nan);                              \
    }
    AWQ_F64_LEVEL(kDppXor1)
    AWQ_F64_LEVEL(kDppXor2)
    AWQ_F64_LEVEL(kDppHalfMirror)
    if (P >= 16) AWQ_F64_LEVEL(kDppMirror)
#undef AWQ_F64_LEVEL
    if (grp < ng && j == 0) {
        double sc, z;
        group_params<AWQ_DTYPE_F64>(nan ? NAN : mn, nan ? NAN : mx, (int)nan, qmin, qmax, sym, sc, z);
        sp_s[grp] = sc;
        sp_z[grp] = z;
        const int64_t gi = r * G + g0 + grp;
        if (scales) scales[gi] = sc != sc ? nan_scale_pick(nan_code, nan != 0) : sw_f32_to_f16((float)sc);
        if (zeros) zeros[gi] = to_i32(z);
    }
    __syncthreads();
    if (qzeros && lane == 0) {
        uint32_t zword = 0;
        for (int g = 0; g < ng; ++g) zword |= (((uint32_t)to_i32(sp_z[g]) - (uint32_t)qmin) & MASK) << (BITS * g);
        qzeros[r * SP + sp] = (int32_t)zword;
    }
    if (!tensor_q && !qweight) return;
    // ---- pass 2: lane = one word of PER elements ----
    const int nwords = (n + PER - 1) / PER;
    for (int c = lane; c < nwords; c += 64) {
        uint32_t wd = 0;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int e = c * PER + i;
            if (e >= n) break;
            const int g = (int)(((float)e + 0.5f) * invL);
            const int32_t q = to_i32(quant1<AWQ_DTYPE_F64>(st[e], sp_s[g], sp_z[g], qmin, qmax));
            if (tensor_q) tensor_q[r * K + span0 + e] = q;
            wd |= (((uint32_t)q - (uint32_t)qmin) & MASK) << (BITS * i);
        }
        if (qweight) qweight[r * wpr + span0 / PER + c] = (int32_t)wd;
    }
}

// Reference _quantize_tensor (awq.py:215-250, mode 0: clamp(round(x / s + z))) and
// _dequantize_tensor (awq.py:252-284, mode 1: (x - z) * s) with caller-given per-group
// parameters, under torch's type promotion (include/awq_hip.h awq_apply_params_ex): the first
// op is evaluated in dtype d1, the second in d2 (= the output's dtype), each in torch's
// per-op way — fp32 math for bf16 / fp16 / fp32 (fp64 for fp64), one rounding to the op's
// dtype; integer ops (mode 1) wrap at their width.  An operand of another dtype is converted
// to the op's dtype first (c10::convert: a float to bf16 / fp16 through fp32; an integer to
// a float dtype as RN_f32 of the exact integer, then RN to bf16 / fp16 — to fp64 directly;
// to an integer dtype by truncation to its width), except a one-element parameter of a
// bf16 / fp16 op under AWQ_APPLY_*_ONE_ELEMENT, which enters at its own value in fp32
// (ATen CPU's original_scalar_value); AWQ_APPLY_IEEE_CLAMP: clamp(-0, 0, qmax) = +0 (torch's GPU
// clamp; its CPU clamp keeps the -0).  Values travel between the steps as exact doubles
// (floats) or exact 64-bit integers (integers; uint64 tensors keep their bits), so int64
// tensors and parameters beyond 2^53 stay exact.  Group g of row r covers elements
// [g L, g L + L) of the row; L = 1 is one parameter per element (any broadcast, expanded by
// the caller).
namespace apply {

enum Op { kDiv, kAdd, kSub, kMul };

struct Val {
    double f;     // kind 0
    int64_t i;    // kind 1 (signed) / 2 (uint64 bits)
    int kind;
};

__device__ __forceinline__ Val of_f(double f) { return Val{f, 0, 0}; }
__device__ __forceinline__ Val of_i(int64_t i, int kind = 1) { return Val{0.0, i, kind}; }
__device__ __forceinline__ bool is_int(int d) { return d >= AWQ_DTYPE_I32; }

__device__ __forceinline__ Val load(const void* x, int dt, int64_t i) {
    switch (dt) {
    case AWQ_DTYPE_BF16: return of_f((double)__uint_as_float((uint32_t)((const uint16_t*)x)[i] << 16));
    case AWQ_DTYPE_F16: return of_f((double)sw_f16_to_f32(((const uint16_t*)x)[i]));
    case AWQ_DTYPE_F32: return of_f((double)((const float*)x)[i]);
    case AWQ_DTYPE_F64: return of_f(((const double*)x)[i]);
    case AWQ_DTYPE_I32: return of_i(((const int32_t*)x)[i]);
    case AWQ_DTYPE_I64: return of_i(((const int64_t*)x)[i]);
    case AWQ_DTYPE_I16: return of_i(((const int16_t*)x)[i]);
    case AWQ_DTYPE_I8: return of_i(((const int8_t*)x)[i]);
    case AWQ_DTYPE_U8: return of_i(((const uint8_t*)x)[i]);
    case AWQ_DTYPE_BOOL: return of_i(((const uint8_t*)x)[i] != 0);
    case AWQ_DTYPE_U16: return of_i(((const uint16_t*)x)[i]);
    case AWQ_DTYPE_U32: return of_i(((const uint32_t*)x)[i]);
    default: return of_i(((const int64_t*)x)[i], 2);    // AWQ_DTYPE_U64
    }
}

// truncation of a 64-bit pattern to integer dtype d (sign- or zero-extended back)
__device__ __forceinline__ int64_t wrap_to(uint64_t v, int d) {
    switch (d) {
    case AWQ_DTYPE_I32: return (int32_t)(uint32_t)v;
    case AWQ_DTYPE_I16: return (int16_t)(uint16_t)v;
    case AWQ_DTYPE_I8: return (int8_t)(uint8_t)v;
    case AWQ_DTYPE_U8: return (uint8_t)v;
    default: return (int64_t)v;
    }
}

// fp32 result of an op rounded to a bf16 / fp16 / fp32 op dtype (a NaN to the dtype's own)
__device__ __forceinline__ float round_to(float r, int d) {
    if (d == AWQ_DTYPE_BF16) return __builtin_isnan(r) ? __uint_as_float(0x7FC00000u) : sw_rn_bf16(r);
    if (d == AWQ_DTYPE_F16) return sw_f16_to_f32(sw_f32_to_f16(r));
    return r;
}

// RN_f32 of an exact integer (int64 or uint64 bits)
__device__ __forceinline__ float int_to_f32(const Val& v) {
    return v.kind == 2 ? (float)(uint64_t)v.i : (float)v.i;
}

// c10::convert of an exactly held value to dtype d
__device__ __forceinline__ Val convert(const Val& v, int d) {
    if (is_int(d)) return of_i(wrap_to(v.kind ? (uint64_t)v.i : (uint64_t)(int64_t)v.f, d));
    if (v.kind == 0) return of_f(d == AWQ_DTYPE_F64 ? v.f : (double)round_to((float)v.f, d));
    if (d == AWQ_DTYPE_F64) return of_f(v.kind == 2 ? (double)(uint64_t)v.i : (double)v.i);
    return of_f((double)round_to(int_to_f32(v), d));
}

// a parameter word (a double, or an int64 / uint64 under AWQ_APPLY_*_INT / _UNSIGNED)
__device__ __forceinline__ Val param(const double* p, int64_t i, bool as_int, bool as_unsigned) {
    if (!as_int) return of_f(p[i]);
    return of_i(__double_as_longlong(p[i]), as_unsigned ? 2 : 1);
}

// a parameter as it enters an op of dtype d
__device__ __forceinline__ Val enter(const Val& v, int d, bool one_element) {
    if (one_element && (d == AWQ_DTYPE_BF16 || d == AWQ_DTYPE_F16))
        return of_f(v.kind ? (double)int_to_f32(v) : (double)(float)v.f);
    return convert(v, d);
}

// a, b already in dtype d
__device__ __forceinline__ Val op(Op o, const Val& a, const Val& b, int d) {
#pragma clang fp contract(off)
    if (is_int(d)) {
        const uint64_t ua = (uint64_t)a.i, ub = (uint64_t)b.i;
        return of_i(wrap_to(o == kSub ? ua - ub : o == kMul ? ua * ub : ua + ub, d));
    }
    if (d == AWQ_DTYPE_F64)
        return of_f(o == kDiv ? a.f / b.f : o == kAdd ? a.f + b.f : o == kSub ? a.f - b.f : a.f * b.f);
    const float fa = (float)a.f, fb = (float)b.f;
    const float r = o == kDiv ? fa / fb : o == kAdd ? fa + fb : o == kSub ? fa - fb : fa * fb;
    return of_f((double)round_to(r, d));
}

__device__ __forceinline__ void store(void* out, int d, int64_t i, const Val& v) {
    switch (d) {
    case AWQ_DTYPE_BF16: ((uint16_t*)out)[i] = (uint16_t)(__float_as_uint((float)v.f) >> 16); break;
    case AWQ_DTYPE_F16: ((uint16_t*)out)[i] = sw_f32_to_f16((float)v.f); break;
    case AWQ_DTYPE_F32: ((float*)out)[i] = (float)v.f; break;
    case AWQ_DTYPE_F64: ((double*)out)[i] = v.f; break;
    case AWQ_DTYPE_I32: ((int32_t*)out)[i] = (int32_t)v.i; break;
    case AWQ_DTYPE_I64: ((int64_t*)out)[i] = v.i; break;
    case AWQ_DTYPE_I16: ((int16_t*)out)[i] = (int16_t)v.i; break;
    case AWQ_DTYPE_I8: ((int8_t*)out)[i] = (int8_t)v.i; break;
    default: ((uint8_t*)out)[i] = (uint8_t)v.i;    // AWQ_DTYPE_U8
    }
}

}  // namespace apply

__global__ __launch_bounds__(256) void awq_apply_kernel(const void* __restrict__ x, int xdt, int64_t rows, int64_t K,
                                                        int64_t L, const double* __restrict__ sp,
                                                        const double* __restrict__ zp, int qmin, int qmax, int mode,
                                                        int d1, int d2, int flags, void* __restrict__ out) {
    using namespace apply;
    const bool s_one = (flags & AWQ_APPLY_SCALE_ONE_ELEMENT) != 0, z_one = (flags & AWQ_APPLY_ZERO_ONE_ELEMENT) != 0;
    const bool s_int = (flags & AWQ_APPLY_SCALE_INT) != 0, z_int = (flags & AWQ_APPLY_ZERO_INT) != 0;
    const bool s_uns = (flags & AWQ_APPLY_SCALE_UNSIGNED) != 0, z_uns = (flags & AWQ_APPLY_ZERO_UNSIGNED) != 0;
    const bool ieee_clamp = (flags & AWQ_APPLY_IEEE_CLAMP) != 0;
    const int64_t G = (K + L - 1) / L;
    const int64_t total = rows * K;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / K, k = i - r * K;
        const int64_t gi = r * G + k / L;
        const Val v = convert(load(x, xdt, i), d1);
        const Val s = param(sp, gi, s_int, s_uns), z = param(zp, gi, z_int, z_uns);
        Val t;
        if (mode == 0) {
            t = op(kDiv, v, enter(s, d1, s_one), d1);                               // awq.py:245
            t = op(kAdd, convert(t, d2), enter(z, d2, z_one), d2);
            t.f = clampq(__builtin_rint(t.f), (double)qmin, (double)qmax);         // awq.py:248
            if (ieee_clamp && t.f == 0.0 && qmin == 0) t.f = 0.0;                   // GPU clamp: +0
        } else {
            t = op(kSub, v, enter(z, d1, z_one), d1);                               // awq.py:282
            t = op(kMul, convert(t, d2), enter(s, d2, s_one), d2);
        }
        store(out, d2, i, t);
    }
}

__global__ __launch_bounds__(256) void awq_pack_kernel(const int32_t* __restrict__ v, int64_t rows,
                                                       int64_t n, int bits, int qmin,
                                                       int32_t* __restrict__ packed) {
    const int per = 32 / bits;
    const uint32_t mask = (1u << bits) - 1u;
    const int64_t words = (n + per - 1) / per;
    const int64_t total = rows * words;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / words, c = i - r * words;
        uint32_t wd = 0;
        for (int j = 0; j < per; ++j) {
            const int64_t k = c * per + j;
            if (k < n) wd |= (((uint32_t)v[r * n + k] - (uint32_t)qmin) & mask) << (bits * j);
        }
        packed[i] = (int32_t)wd;
    }
}

// awq.py:459-539: dq = fp16(fp16(q - z) * s) stored fp32; q/z from int32 arrays or packed.
__global__ __launch_bounds__(256) void awq_dequant_kernel(
    const int32_t* __restrict__ tensor_q, const int32_t* __restrict__ qweight,
    const uint16_t* __restrict__ scales, const int32_t* __restrict__ zeros,
    const int32_t* __restrict__ qzeros, int64_t rows, int64_t K, int64_t L, int bits, int qmin,
    float* __restrict__ out) {
    const int64_t G = (K + L - 1) / L;
    const int per = 32 / bits;
    const uint32_t mask = (1u << bits) - 1u;
    const int64_t wpr = (K + per - 1) / per, zpr = (G + per - 1) / per;
    const int64_t total = rows * K;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / K, k = i - r * K, g = k / L;
        int32_t q, z;
        if (tensor_q) {
            q = tensor_q[i];
            z = zeros[r * G + g];
        } else {
            q = (int32_t)((((uint32_t)qweight[r * wpr + k / per]) >> (bits * (k % per))) & mask) + qmin;
            z = (int32_t)((((uint32_t)qzeros[r * zpr + g / per]) >> (bits * (g % per))) & mask) + qmin;
        }
        const int32_t diff = (int32_t)((uint32_t)q - (uint32_t)z);
        const float h = sw_f16_to_f32(sw_f32_to_f16((float)diff));
        const float s = sw_f16_to_f32(scales[r * G + g]);
        const uint16_t d16 = sw_f32_to_f16(h * s);
        float v = sw_f16_to_f32(d16);
        if (v != v) v = __uint_as_float(dq_nan_bits(d16, k - g * L, min(L, K - g * L)));
        out[i] = v;
    }
}

// awq_dequantize_packed for word-aligned groups (K % PER == 0, L % PER == 0; PER = 32 / bits):
// one thread per qweight word — its PER elements share one row and one group — so one
// division per word instead of three per element, one scale and one qzeros load per word,
// and the PER fp32 outputs leave as 16-B stores.  Arithmetic (awq.py:459-539): q - z is an
// integer of at most 8 bits, exact in fp16; h * s of that integer and an fp16 scale needs
// at most 19 significand bits, so the f32 product is exact and one hardware RNE conversion
// to fp16 gives RN_f16(h * s) bit for bit (NaN lanes take the software conversion, which
// keeps the payload as torch does).  Memory-bound: 0.5 B (4-bit) read + 4 B written per element.
#ifdef AWQ_DIAG   // round-2/3 dequantize variants: A/B builds only (scripts/, make diag)
template <int BITS>
__global__ __launch_bounds__(256) void awq_dequant_words_kernel(
    const int32_t* __restrict__ qweight, const uint16_t* __restrict__ scales, const int32_t* __restrict__ qzeros,
    int64_t words, uint32_t wpr, uint32_t L, uint32_t G, uint32_t zpr, int qmin, float* __restrict__ out, float /*invL*/) {
    constexpr int PER = 32 / BITS;
    constexpr uint32_t MASK = (1u << BITS) - 1u;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= words) return;
    int64_t r;
    uint32_t c;
    if (words <= (int64_t)0xFFFFFFFFu) {                 // 32-bit index arithmetic
        const uint32_t r32 = (uint32_t)i / wpr;
        r = r32;
        c = (uint32_t)i - r32 * wpr;
    } else {
        r = i / wpr;
        c = (uint32_t)(i - r * wpr);
    }
    const uint32_t g = (uint32_t)(((uint64_t)c * PER) / L);   // (64-bit: c * PER may pass 2^32)
    const uint32_t wq = (uint32_t)__builtin_nontemporal_load(qweight + i);
    const float s = (float)__builtin_bit_cast(_Float16, scales[r * G + g]);
    const int32_t z = (int32_t)(((uint32_t)qzeros[r * zpr + g / PER] >> (BITS * (g % PER))) & MASK) + qmin;
    float v[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int32_t q = (int32_t)((wq >> (BITS * j)) & MASK) + qmin;
        const float p = (float)(q - z) * s;
        if (__builtin_expect(__builtin_isnan(p), 0)) {   // NaN bits of the reference's fp32 copy
            const int64_t k = (int64_t)c * PER + j, K = (int64_t)wpr * PER, g0 = (int64_t)g * L;
            v[j] = __uint_as_float(dq_nan_bits(sw_f32_to_f16(p), k - g0, min((int64_t)L, K - g0)));
        } else {
            v[j] = (float)(_Float16)p;
        }
    }
    typedef float f4 __attribute__((ext_vector_type(4)));
    f4* o = (f4*)(out + i * PER);
#pragma unroll
    for (int j = 0; j < PER / 4; ++j) {
        const f4 t = {v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]};
        __builtin_nontemporal_store(t, o + j);
    }
}

// The same, with the two memory-side fixes the round-2 PMC asked for (profiles/round2/r2as:
// 1.15x algorithmic reads, 1.13x writes):
//  * writes: a 4-bit thread's 8 fp32 results (32 B) went out as two 16-B stores 32 B apart,
//    so every store instruction half-covered 2 KiB of 64-B lines; here the block's 8 KiB of
//    results are staged in LDS and each store instruction of a wave writes 1 KiB contiguous
//    (16 B per lane);
//  * reads: consecutive blocks (neighbouring words of a row, which share the row's scale and
//    qzeros lines) were dealt round-robin over the 8 XCDs, each XCD's L2 fetching the shared
//    lines again; blocks are renumbered so each XCD takes a contiguous range of the words.
constexpr int kDqThreads = 256;

__device__ __forceinline__ uint32_t xcd_contiguous_block(uint32_t b, uint32_t nb) {
    const uint32_t full = nb / 8u * 8u;           // blocks b are dealt to XCD b % 8
    if (b >= full) return b;
    return (b % 8u) * (full / 8u) + b / 8u;       // XCD x: blocks x * full/8 .. (x+1) * full/8 - 1
}

template <int BITS, bool REMAP>
__global__ __launch_bounds__(kDqThreads) void awq_dequant_words_v2_kernel(
    const int32_t* __restrict__ qweight, const uint16_t* __restrict__ scales, const int32_t* __restrict__ qzeros,
    int64_t words, uint32_t wpr, uint32_t L, uint32_t G, uint32_t zpr, int qmin, float* __restrict__ out, float /*invL*/) {
    constexpr int PER = 32 / BITS;
    constexpr uint32_t MASK = (1u << BITS) - 1u;
    __shared__ __attribute__((aligned(16))) float stage[kDqThreads * PER];
    const int64_t blk = REMAP ? xcd_contiguous_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const int64_t w0 = blk * kDqThreads;
    const int64_t i = w0 + threadIdx.x;
    float v[PER];
    if (i < words) {
        int64_t r;
        uint32_t c;
        if (words <= (int64_t)0xFFFFFFFFu) {
            const uint32_t r32 = (uint32_t)i / wpr;
            r = r32;
            c = (uint32_t)i - r32 * wpr;
        } else {
            r = i / wpr;
            c = (uint32_t)(i - r * wpr);
        }
        const uint32_t g = (uint32_t)(((uint64_t)c * PER) / L);
        const uint32_t wq = (uint32_t)__builtin_nontemporal_load(qweight + i);
        const float s = (float)__builtin_bit_cast(_Float16, scales[r * G + g]);
        const int32_t z = (int32_t)(((uint32_t)qzeros[r * zpr + g / PER] >> (BITS * (g % PER))) & MASK) + qmin;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int32_t q = (int32_t)((wq >> (BITS * j)) & MASK) + qmin;
            const float p = (float)(q - z) * s;
            if (__builtin_expect(__builtin_isnan(p), 0)) {   // NaN bits of the reference's fp32 copy
                const int64_t k = (int64_t)c * PER + j, K = (int64_t)wpr * PER, g0 = (int64_t)g * L;
                v[j] = __uint_as_float(dq_nan_bits(sw_f32_to_f16(p), k - g0, min((int64_t)L, K - g0)));
            } else {
                v[j] = (float)(_Float16)p;
            }
        }
    }
    typedef float f4 __attribute__((ext_vector_type(4)));
    const int64_t nw = min((int64_t)kDqThreads, words - w0);       // words of this block
    if (PER == 4 || nw < kDqThreads) {
        // 8-bit (16 B per thread: one contiguous 1 KiB per wave instruction already) and the
        // grid's partial last block: direct stores
        if (i < words) {
            f4* o = (f4*)(out + i * PER);
#pragma unroll
            for (int j = 0; j < PER / 4; ++j)
                __builtin_nontemporal_store((f4){v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]}, o + j);
        }
        return;
    }
    // 4-bit: stage the block's 8 KiB, then lane t of the block stores bytes 16 t + 4 KiB h
#pragma unroll
    for (int j = 0; j < PER / 4; ++j)
        *(f4*)(stage + PER * threadIdx.x + 4 * j) = (f4){v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]};
    __syncthreads();
    f4* o = (f4*)(out + w0 * PER);
#pragma unroll
    for (int h = 0; h < PER / 4; ++h)
        __builtin_nontemporal_store(*(const f4*)(stage + 4 * (threadIdx.x + kDqThreads * h)),
                                    o + threadIdx.x + kDqThreads * h);
}

// The same arithmetic with four outputs per lane: a 4-bit word is shared by two neighbouring
// lanes (each converts one nibble half), so every lane issues exactly one 16-B store and a
// wave's store instruction covers 1 KiB contiguous with no LDS round trip or barrier (v2's
// staging); the word, scale and qzeros loads of the lane pair hit the same dwords.  REMAP: the
// XCD-contiguous block order of v2.
template <int BITS, bool REMAP>
__global__ __launch_bounds__(256) void awq_dequant_quads_kernel(
    const int32_t* __restrict__ qweight, const uint16_t* __restrict__ scales, const int32_t* __restrict__ qzeros,
    int64_t words, uint32_t wpr, uint32_t L, uint32_t G, uint32_t zpr, int qmin, float* __restrict__ out, float /*invL*/) {
    constexpr int PER = 32 / BITS;
    constexpr int LPW = PER / 4;                        // lanes per word: 2 (4-bit), 1 (8-bit)
    constexpr uint32_t MASK = (1u << BITS) - 1u;
    const int64_t blk = REMAP ? xcd_contiguous_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const int64_t t = blk * 256 + threadIdx.x;
    const int64_t i = t / LPW;                          // word
    const int half = (int)(t - i * LPW);                // which 4 fields of the word
    if (i >= words) return;
    int64_t r;
    uint32_t c;
    if (words <= (int64_t)0xFFFFFFFFu) {
        const uint32_t r32 = (uint32_t)i / wpr;
        r = r32;
        c = (uint32_t)i - r32 * wpr;
    } else {
        r = i / wpr;
        c = (uint32_t)(i - r * wpr);
    }
    const uint32_t g = (uint32_t)(((uint64_t)c * PER) / L);
    const uint32_t wq = (uint32_t)__builtin_nontemporal_load(qweight + i) >> (16 * half);
    const float s = (float)__builtin_bit_cast(_Float16, scales[r * G + g]);
    const int32_t z = (int32_t)(((uint32_t)qzeros[r * zpr + g / PER] >> (BITS * (g % PER))) & MASK) + qmin;
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int32_t q = (int32_t)((wq >> (BITS * j)) & MASK) + qmin;
        const float p = (float)(q - z) * s;
        if (__builtin_expect(__builtin_isnan(p), 0)) {   // NaN bits of the reference's fp32 copy
            const int64_t k = (int64_t)c * PER + 4 * half + j, K = (int64_t)wpr * PER, g0 = (int64_t)g * L;
            v[j] = __uint_as_float(dq_nan_bits(sw_f32_to_f16(p), k - g0, min((int64_t)L, K - g0)));
        } else {
            v[j] = (float)(_Float16)p;
        }
    }
    typedef float f4 __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store((f4){v[0], v[1], v[2], v[3]}, (f4*)(out + 4 * t));
}

#endif  // AWQ_DIAG

// Batched four-output lanes: each thread converts U quads (4 outputs, one 16-B store each) of
// its block's 256 * U consecutive quads, with every load of the U quads (qweight word, scale,
// qzeros word) issued before the first conversion — U independent loads in flight per lane
// instead of one, and U times fewer waves (the one-quad kernels are bound by wave turnover:
// one load round trip per short-lived wave).  RUN > 0: RUN consecutive blocks run on one XCD
// (blocks are dealt round-robin over the 8 XCDs) so the scale and qzeros lines a run shares
// are fetched by one L2 — without v2's one-range-per-XCD order, whose 8 concurrent streams
// sit a power-of-two distance apart.
__device__ __forceinline__ uint32_t dq_run_block(uint32_t b, uint32_t nb, uint32_t R) {
    const uint32_t full = nb / (8u * R) * (8u * R);
    if (b >= full) return b;
    const uint32_t x = b % 8u, i = b / 8u;
    return (i / R) * (8u * R) + x * R + (i % R);
}

// Group index e / L of column e by a float estimate and one correction step each way
// (exact for e < 2^22: the estimate is within 1; the launcher admits K < 2^22 for GMODE > 0).
__device__ __forceinline__ uint32_t dq_gdiv(uint32_t e, uint32_t L, float invL) {
    uint32_t q = (uint32_t)((float)e * invL);
    if (q * L > e) --q;
    else if ((q + 1) * L <= e) ++q;
    return q;
}

// GMODE: 0 = a qweight word's PER elements share one group (L % PER == 0); 1 = a quad's 4
// elements do (L % 4 == 0); 2 = any L >= 4 (a quad meets at most two groups: the first
// `bnd` elements take group A's parameters, the rest group B's).  Dequantize of any group
// size at the batched kernel's memory structure (round 4: the per-element generic kernel ran
// group size 100 at 0.10 of 8 TB/s).
template <int BITS, int U, int RUN, int GMODE>
__global__ __launch_bounds__(256) void awq_dequant_batch_kernel(
    const int32_t* __restrict__ qweight, const uint16_t* __restrict__ scales, const int32_t* __restrict__ qzeros,
    int64_t words, uint32_t wpr, uint32_t L, uint32_t G, uint32_t zpr, int qmin, float* __restrict__ out,
    float invL) {
    constexpr int PER = 32 / BITS;
    constexpr int LPW = PER / 4;                        // lanes (quads) per word
    constexpr uint32_t MASK = (1u << BITS) - 1u;
    const int64_t blk = RUN > 0 ? dq_run_block(blockIdx.x, gridDim.x, RUN) : blockIdx.x;
    const int64_t quads = words * LPW;
    const int64_t q0 = blk * (256 * U) + threadIdx.x;
    uint32_t wq[U], zq[U], zq2[U];
    uint16_t sb[U], sb2[U];
    int64_t ii[U];
    uint32_t cc[U], gg[U], gg2[U], bnd[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const int64_t q = min(q0 + 256 * k, quads - 1);   // (past the end: a valid address, no store)
        const int64_t i = q / LPW;
        int64_t r;
        uint32_t c;
        if (words <= (int64_t)0xFFFFFFFFu) {
            const uint32_t r32 = (uint32_t)i / wpr;
            r = r32;
            c = (uint32_t)i - r32 * wpr;
        } else {
            r = i / wpr;
            c = (uint32_t)(i - r * wpr);
        }
        uint32_t g, g2 = 0, b = 4;
        if constexpr (GMODE == 0) {
            g = (uint32_t)(((uint64_t)c * PER) / L);
        } else {
            const uint32_t e0 = c * PER + 4u * (uint32_t)(q - i * LPW);
            g = dq_gdiv(e0, L, invL);
            if constexpr (GMODE == 2) {
                b = min((g + 1) * L - e0, 4u);
                g2 = b < 4 ? g + 1 : g;
            }
        }
        ii[k] = i;
        cc[k] = c;
        gg[k] = g;
        wq[k] = (uint32_t)qweight[i];   // plain load: an nt load bypasses a cache-resident input (r5d1)
        sb[k] = scales[r * G + g];
        zq[k] = (uint32_t)qzeros[r * zpr + g / PER];
        if constexpr (GMODE == 2) {
            gg2[k] = g2;
            bnd[k] = b;
            sb2[k] = scales[r * G + g2];
            zq2[k] = (uint32_t)qzeros[r * zpr + g2 / PER];
        }
    }
    typedef float f4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const int64_t q = q0 + 256 * k;
        if (q >= quads) break;
        const int half = (int)(q - ii[k] * LPW);
        const uint32_t w = wq[k] >> (16 * half);
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool a = GMODE != 2 || (uint32_t)j < bnd[k];
            const uint32_t g = a ? gg[k] : gg2[k];
            const float s = (float)__builtin_bit_cast(_Float16, a ? sb[k] : sb2[k]);
            const int32_t z = (int32_t)(((a ? zq[k] : zq2[k]) >> (BITS * (g % PER))) & MASK) + qmin;
            const int32_t qv = (int32_t)((w >> (BITS * j)) & MASK) + qmin;
            const float p = (float)(qv - z) * s;
            if (__builtin_expect(__builtin_isnan(p), 0)) {   // NaN bits of the reference's fp32 copy
                const int64_t kk = (int64_t)cc[k] * PER + 4 * half + j, K = (int64_t)wpr * PER,
                              g0 = (int64_t)g * L;
                v[j] = __uint_as_float(dq_nan_bits(sw_f32_to_f16(p), kk - g0, min((int64_t)L, K - g0)));
            } else {
                v[j] = (float)(_Float16)p;
            }
        }
        __builtin_nontemporal_store((f4){v[0], v[1], v[2], v[3]}, (f4*)(out + 4 * q));
    }
}

template <int B> constexpr auto dq_batch4_run = awq_dequant_batch_kernel<B, 4, 4, 0>;
template <int B> constexpr auto dq_batch4_run_q = awq_dequant_batch_kernel<B, 4, 4, 1>;
template <int B> constexpr auto dq_batch4_run_e = awq_dequant_batch_kernel<B, 4, 4, 2>;
constexpr int kDqDefault = 8;   // batched lanes in XCD runs: profiles/round3/dequant
#ifdef AWQ_DIAG
template <int B> constexpr auto dq_v2_remap = awq_dequant_words_v2_kernel<B, true>;
template <int B> constexpr auto dq_v2_plain = awq_dequant_words_v2_kernel<B, false>;
template <int B> constexpr auto dq_quads_plain = awq_dequant_quads_kernel<B, false>;
template <int B> constexpr auto dq_quads_remap = awq_dequant_quads_kernel<B, true>;
template <int B> constexpr auto dq_batch4 = awq_dequant_batch_kernel<B, 4, 0, 0>;
template <int B> constexpr auto dq_batch8 = awq_dequant_batch_kernel<B, 8, 0, 0>;
template <int B> constexpr auto dq_batch8_run = awq_dequant_batch_kernel<B, 8, 2, 0>;
template <int B> constexpr auto dq_batch2_run = awq_dequant_batch_kernel<B, 2, 4, 0>;
template <int B> constexpr auto dq_batch1_run = awq_dequant_batch_kernel<B, 1, 4, 0>;
template <int B> constexpr auto dq_batch2 = awq_dequant_batch_kernel<B, 2, 0, 0>;
template <int B> constexpr auto dq_batch2_run8 = awq_dequant_batch_kernel<B, 2, 8, 0>;
#endif

// Measurement helper (awq_dequant_ceiling): the batched dequantize's memory structure without its
// arithmetic and parameter loads — per quad one 4-B nt load of the packed word (a lane pair
// shares it) and one 16-B nt store (1 KiB per wave instruction), U quads per lane with the loads
// issued first: read 1 : write 8, the 4-bit dequantize's ratio.
template <int U>
__global__ __launch_bounds__(256) void awq_dequant_ceiling_kernel(const uint32_t* __restrict__ words,
                                                                  float* __restrict__ out, int64_t quads) {
    const int64_t q0 = (int64_t)blockIdx.x * (256 * U) + threadIdx.x;
    uint32_t w[U];
#pragma unroll
    for (int k = 0; k < U; ++k) w[k] = __builtin_nontemporal_load(words + min(q0 + 256 * k, quads - 1) / 2);
    typedef float f4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const int64_t q = q0 + 256 * k;
        if (q >= quads) break;
        const uint32_t v = w[k] >> (16 * (int)(q & 1));
        const f4 o = {(float)(v & 15u), (float)((v >> 4) & 15u), (float)((v >> 8) & 15u), (float)((v >> 12) & 15u)};
        __builtin_nontemporal_store(o, (f4*)(out + 4 * q));
    }
}

inline unsigned grid_for(int64_t work, int64_t per_block, int64_t cap) {
    int64_t b = (work + per_block - 1) / per_block;
    if (b < 1) b = 1;
    if (b > cap) b = cap;
    return (unsigned)b;
}

}  // namespace

hipError_t launch_generic(const void* w, int dtype, int64_t rows, int64_t K, int64_t L, int bits,
                          int symmetric, int32_t* tensor_q, uint16_t* scales, int32_t* zeros,
                          int32_t* qweight, int32_t* qzeros, hipStream_t stream, bool small, int n_grid,
                          int n_cand, double* s_exact, double* z_exact, bool torch_gpu) {
    if (torch_gpu && (n_cand > 0 || tensor_q || scales || zeros || qweight || qzeros))
        return hipErrorInvalidValue;   // (torch's GPU semantics: the exact-parameter outputs only)
    const int qmin = symmetric ? -(1 << (bits - 1)) : 0;
    const int qmax = symmetric ? (1 << (bits - 1)) - 1 : (1 << bits) - 1;
    const int per = 32 / bits;
    const int64_t G = (K + L - 1) / L;
    const unsigned grid = grid_for(rows * ((G + per - 1) / per), 4, 256 * 16);
    const bool search = n_cand > 0;
    // fp64 spans: the LDS span wherever the span fits 16 KiB (3.2-3.7 TB/s of input at gs 64 /
    // 128, against the register span's 1.4-2.4: profiles/round3/r3n), else the strided span.
    // Diagnostics builds (AWQ_DIAG, tuning gen_noreg): 1 = the strided span only, 2 = the
    // register span at gs 64 / 128
#ifdef AWQ_DIAG
    const int f64_span = tuning().gen_noreg;
    if (dtype == AWQ_DTYPE_F64 && !search && !s_exact && !z_exact && (L == 64 || L == 128) && f64_span == 2) {
        const unsigned blocks = (unsigned)((rows * ((G + per - 1) / per) + 3) / 4);
        const double* wd = (const double*)w;
#define AWQ_SPAN_REG(LPI, PER)                                                                              \
        hipLaunchKernelGGL((awq_generic_span_reg_kernel<LPI, PER>), dim3(blocks), dim3(256), 0, stream, wd, rows, K, \
                           qmin, qmax, symmetric, nan_scale_code(AWQ_DTYPE_F64, symmetric, small), tensor_q,     \
                           scales, zeros, qweight, qzeros)
        if (L == 64) {
            if (per == 8) AWQ_SPAN_REG(1, 8); else AWQ_SPAN_REG(1, 4);
        } else {
            if (per == 8) AWQ_SPAN_REG(2, 8); else AWQ_SPAN_REG(2, 4);
        }
#undef AWQ_SPAN_REG
        return hipPeekAtLastError();
    }
#else
    constexpr int f64_span = 0;
#endif
    if (dtype == AWQ_DTYPE_F64 && !search && !s_exact && !z_exact && L >= 2 && per * L * 8 <= 16384 &&
        f64_span != 1) {
        const int64_t SP = (G + per - 1) / per;
        const size_t lds = (size_t)(per * L * 8);
        const float invL = 1.0f / (float)L;
        const uint32_t nc = nan_scale_code(AWQ_DTYPE_F64, symmetric, small);
        if (per == 8)
            hipLaunchKernelGGL(awq_f64_span_lds_kernel<8>, dim3((unsigned)(rows * SP)), dim3(64), lds, stream,
                               (const double*)w, rows, K, L, invL, qmin, qmax, symmetric, nc, tensor_q, scales, zeros,
                               qweight, qzeros);
        else
            hipLaunchKernelGGL(awq_f64_span_lds_kernel<4>, dim3((unsigned)(rows * SP)), dim3(64), lds, stream,
                               (const double*)w, rows, K, L, invL, qmin, qmax, symmetric, nc, tensor_q, scales, zeros,
                               qweight, qzeros);
        return hipPeekAtLastError();
    }
    const int smallf = (small ? 1 : 0) | (torch_gpu ? 2 : 0);   // kernel flags: bit 1 = torch's GPU semantics
#define AWQ_GEN(D)                                                                                   \
    do {                                                                                             \
        if (search)                                                                                  \
            hipLaunchKernelGGL((awq_generic_kernel<D, true>), dim3(grid), dim3(256), 0, stream, w, rows, \
                               K, L, bits, qmin, qmax, symmetric, smallf, n_grid, n_cand, tensor_q,   \
                               scales, zeros, qweight, qzeros, s_exact, z_exact);                      \
        else                                                                                         \
            hipLaunchKernelGGL((awq_generic_kernel<D, false>), dim3(grid), dim3(256), 0, stream, w,     \
                               rows, K, L, bits, qmin, qmax, symmetric, smallf, 1, 0, tensor_q, scales, \
                               zeros, qweight, qzeros, s_exact, z_exact);                              \
    } while (0)
    switch (dtype) {
    case AWQ_DTYPE_BF16: AWQ_GEN(AWQ_DTYPE_BF16); break;
    case AWQ_DTYPE_F16: AWQ_GEN(AWQ_DTYPE_F16); break;
    case AWQ_DTYPE_F32: AWQ_GEN(AWQ_DTYPE_F32); break;
    case AWQ_DTYPE_F64: AWQ_GEN(AWQ_DTYPE_F64); break;
    default: return hipErrorInvalidValue;
    }
#undef AWQ_GEN
    return hipPeekAtLastError();
}

hipError_t launch_apply(const void* x, int xdt, int64_t rows, int64_t K, int64_t L, const double* scales,
                        const double* zeros, int qmin, int qmax, int mode, int d1, int d2, int flags, void* out,
                        hipStream_t stream) {
    const int64_t total = rows * K;
    if (total <= 0) return hipSuccess;
    hipLaunchKernelGGL(awq_apply_kernel, dim3(grid_for(total, 256, 256 * 16)), dim3(256), 0, stream, x, xdt, rows, K,
                       L, scales, zeros, qmin, qmax, mode, d1, d2, flags, out);
    return hipPeekAtLastError();
}

hipError_t launch_dequant_ceiling(const void* words, void* out, int64_t out_bytes, hipStream_t stream) {
    const int64_t quads = out_bytes / 16;
    if (quads <= 0) return hipSuccess;
    hipLaunchKernelGGL(awq_dequant_ceiling_kernel<2>, dim3((unsigned)((quads + 511) / 512)), dim3(256), 0, stream,
                       (const uint32_t*)words, (float*)out, quads);
    return hipPeekAtLastError();
}

hipError_t launch_pack(const int32_t* v, int64_t rows, int64_t n, int bits, int qmin,
                       int32_t* packed, hipStream_t stream) {
    const int per = 32 / bits;
    const int64_t total = rows * ((n + per - 1) / per);
    if (total <= 0) return hipSuccess;
    hipLaunchKernelGGL(awq_pack_kernel, dim3(grid_for(total, 256, 256 * 16)), dim3(256), 0, stream, v,
                       rows, n, bits, qmin, packed);
    return hipPeekAtLastError();
}

hipError_t launch_dequant(const int32_t* tensor_q, const int32_t* qweight, const uint16_t* scales,
                          const int32_t* zeros, const int32_t* qzeros, int64_t rows, int64_t K,
                          int64_t L, int bits, int qmin, float* out, hipStream_t stream) {
    const int64_t total = rows * K;
    if (total <= 0) return hipSuccess;
    const int per = 32 / bits;
    const int64_t G = (K + L - 1) / L;
    // the batched quad kernel: word-aligned groups (GMODE 0), quad-aligned (1), or any L >= 4 (2)
    // for rows of < 2^22 elements
    const int gmode = L % per == 0 ? 0 : (L % 4 == 0 ? 1 : 2);
    if (!tensor_q && K % per == 0 && (gmode == 0 || (L >= 4 && K < ((int64_t)1 << 22))) &&
        ((uintptr_t)out & 15) == 0 && K / per <= 0x7FFFFFFF &&
        L <= 0x7FFFFFFF && G <= 0x7FFFFFFF && total / per < ((int64_t)1 << 32) - 256) {   // one thread per word
        const int64_t words = total / per;
        const uint32_t wpr = (uint32_t)(K / per), zpr = (uint32_t)((G + per - 1) / per);
        const dim3 grid((unsigned)((words + 255) / 256)), block(256);
        // the batched four-output lanes in XCD runs (kDqDefault = 8).  Diagnostics builds
        // (AWQ_DIAG, awq_diag.h dq_words_v1) also reach the A/B variants: 1 round-2 word
        // kernel, 2 / 3 LDS-staged v2 with / without XCD-contiguous blocks, 4 / 5 four-output
        // lanes without / with XCD-contiguous blocks, 6 / 7 batched lanes (4 / 8 quads), 9 the
        // batched lanes in XCD runs of 2 blocks
        int v = kDqDefault;
        const float invL = 1.0f / (float)L;
#ifdef AWQ_DIAG
        if (gmode == 0 && tuning().dq_words_v1 > 0 && tuning().dq_words_v1 <= 13) v = tuning().dq_words_v1;
#endif
#define AWQ_DQ(KER, GRID)                                                                                   \
        do {                                                                                                \
            if (bits == 4)                                                                                  \
                hipLaunchKernelGGL(KER<4>, GRID, block, 0, stream, qweight, scales, qzeros, words, wpr,     \
                                   (uint32_t)L, (uint32_t)G, zpr, qmin, out, invL);                         \
            else                                                                                            \
                hipLaunchKernelGGL(KER<8>, GRID, block, 0, stream, qweight, scales, qzeros, words, wpr,     \
                                   (uint32_t)L, (uint32_t)G, zpr, qmin, out, invL);                         \
        } while (0)
        const dim3 grid_q((unsigned)((words * (per / 4) + 255) / 256));
        const dim3 grid_b4((unsigned)((words * (per / 4) + 1023) / 1024)),
            grid_b8((unsigned)((words * (per / 4) + 2047) / 2048));
        switch (v) {
#ifdef AWQ_DIAG
        case 10: AWQ_DQ(dq_batch2_run, dim3((unsigned)((words * (per / 4) + 511) / 512))); break;
        case 11: AWQ_DQ(dq_batch1_run, grid_q); break;
        case 12: AWQ_DQ(dq_batch2, dim3((unsigned)((words * (per / 4) + 511) / 512))); break;
        case 13: AWQ_DQ(dq_batch2_run8, dim3((unsigned)((words * (per / 4) + 511) / 512))); break;
        case 6: AWQ_DQ(dq_batch4, grid_b4); break;
        case 7: AWQ_DQ(dq_batch8, grid_b8); break;
        case 9: AWQ_DQ(dq_batch8_run, grid_b8); break;
        case 1: AWQ_DQ(awq_dequant_words_kernel, grid); break;
        case 2: AWQ_DQ(dq_v2_remap, grid); break;
        case 3: AWQ_DQ(dq_v2_plain, grid); break;
        case 4: AWQ_DQ(dq_quads_plain, grid_q); break;
        case 5: AWQ_DQ(dq_quads_remap, grid_q); break;
#endif
        default:
            if (gmode == 0) AWQ_DQ(dq_batch4_run, grid_b4);
            else if (gmode == 1) AWQ_DQ(dq_batch4_run_q, grid_b4);
            else AWQ_DQ(dq_batch4_run_e, grid_b4);
            break;
        }
#undef AWQ_DQ
        return hipPeekAtLastError();
    }
    hipLaunchKernelGGL(awq_dequant_kernel, dim3(grid_for(total, 256, 256 * 16)), dim3(256), 0, stream,
                       tensor_q, qweight, scales, zeros, qzeros, rows, K, L, bits, qmin, out);
    return hipPeekAtLastError();
}

}  // namespace awq
