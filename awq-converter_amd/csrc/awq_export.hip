// awq_export.hip — AutoAWQ "GEMM" layout export of packed 4-bit results (SURVEY.md §8f
// row 4; no reference counterpart: the reference emits unpacked int32 only).
//
// Input: this library's row-major packed outputs of a [N = out_features, K = in_features]
// weight: qweight int32 [N, K/8] (nibble j of word c = element 8c+j, value q - qmin),
// qzeros int32 [N, G/8] (same packing of the zero points), scales fp16 [N, G].
// Output, the layout AutoAWQ's WQLinear_GEMM kernels read (K-major, packed along N with
// the interleave AWQ_ORDER = [0, 2, 4, 6, 1, 3, 5, 7]: nibble i of output word c holds
// column 8c + AWQ_ORDER[i]):
//   qweight_t int32 [K, N/8], qzeros_t int32 [G, N/8], scales_t fp16 [G, N].
// Values are unchanged (unsigned fields, dq = (q - z) * s as AutoAWQ dequantizes).
//
// qweight: one workgroup per 256 (n) x 256 (k) nibble tile, an in-register 8 x 8 nibble
// transpose and an LDS-staged store (both HBM sides in 128-B row pieces); scales / qzeros:
// one workgroup per 64 (n) x 32 (g) tile through LDS.  HBM-bound, about 1 B/element.
#include "awq_internal.h"

namespace awq {
namespace {

#ifndef AWQ_EXPORT_NT_MIN
// qweight exports of at least this many bytes are stored nontemporal (past the caches:
// larger than half the 256 MB MALL they only evict; smaller ones gain from write-back)
#define AWQ_EXPORT_NT_MIN (128ll << 20)
#endif
// qweight: a 256 (n) x 256 (k) nibble tile per workgroup.  A lane holds the words of 8
// consecutive rows (8 nb .. 8 nb + 7) at one k-word kw, takes them in AWQ_ORDER (register
// renaming) and transposes the 8 x 8 nibble matrix in registers (three rounds of masked
// swaps): word j is then output word (k = 8 kw + j, column nb).  Loads: 16 B per lane (8
// lanes per 128-B row piece; 4-B loads when K % 32 != 0).  The words are staged in LDS with
// the column XOR-swizzled by kw (2-way writes, the minimum for 64 lanes) and stored as 16-B
// pieces of 128-B output rows.
constexpr int kT2 = 256;                 // tile edge in nibbles (n and k)
__device__ __forceinline__ void swapn(uint32_t& x, uint32_t& y, int sh, uint32_t mask) {
    const uint32_t t = ((x >> sh) ^ y) & mask;
    x ^= t << sh;
    y ^= t;
}
// rows a[0..7] (8 nibbles each) -> b[j] = nibble j of every row, row AWQ_ORDER[i] at nibble i
__device__ __forceinline__ void nibble_transpose8(const uint32_t (&a)[8], uint32_t (&b)[8]) {
    b[0] = a[0]; b[1] = a[2]; b[2] = a[4]; b[3] = a[6];
    b[4] = a[1]; b[5] = a[3]; b[6] = a[5]; b[7] = a[7];
#pragma unroll
    for (int i = 0; i < 4; ++i) swapn(b[i], b[i + 4], 16, 0x0000FFFFu);
#pragma unroll
    for (int i = 0; i < 8; i += 4) {
        swapn(b[i], b[i + 2], 8, 0x00FF00FFu);
        swapn(b[i + 1], b[i + 3], 8, 0x00FF00FFu);
    }
#pragma unroll
    for (int i = 0; i < 8; i += 2) swapn(b[i], b[i + 1], 4, 0x0F0F0F0Fu);
}
__device__ __forceinline__ void transpose_to_lds(const uint32_t (&a)[8], uint32_t (*ob)[kT2 / 8], int kw, int nb) {
    uint32_t b[8];
    nibble_transpose8(a, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) ob[8 * kw + j][nb ^ kw] = b[j];
}
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <bool VEC, bool NT>
__global__ __launch_bounds__(256) void awq_export_qweight_kernel(const int32_t* __restrict__ qweight, int64_t N,
                                                                    int64_t K, int32_t* __restrict__ qweight_t) {
    __shared__ uint32_t ob[kT2][kT2 / 8];                 // [k in tile][output word column], swizzled
    const int64_t n0 = (int64_t)blockIdx.x * kT2, k0 = (int64_t)blockIdx.y * kT2;
    const int64_t wpr = K / 8, wpr_t = N / 8;
    const int t = threadIdx.x;
    if constexpr (VEC) {
        // K % 32 == 0, 16-B aligned rows: lanes (kq = t & 7, nb = t >> 3) read 16 B each, 8
        // lanes per 128-B row piece
        const int kq = t & 7, nb = t >> 3;
        const int64_t kwg = k0 / 8 + 4 * kq;
        uint4 v[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const int64_t n = n0 + 8 * nb + r;
            v[r] = make_uint4(0, 0, 0, 0);
            if (n < N && kwg < wpr) {
                v[r] = *(const uint4*)(qweight + n * wpr + kwg);
            }
        }
        const uint32_t a0[8] = {v[0].x, v[1].x, v[2].x, v[3].x, v[4].x, v[5].x, v[6].x, v[7].x};
        const uint32_t a1[8] = {v[0].y, v[1].y, v[2].y, v[3].y, v[4].y, v[5].y, v[6].y, v[7].y};
        const uint32_t a2[8] = {v[0].z, v[1].z, v[2].z, v[3].z, v[4].z, v[5].z, v[6].z, v[7].z};
        const uint32_t a3[8] = {v[0].w, v[1].w, v[2].w, v[3].w, v[4].w, v[5].w, v[6].w, v[7].w};
        transpose_to_lds(a0, ob, 4 * kq + 0, nb);
        transpose_to_lds(a1, ob, 4 * kq + 1, nb);
        transpose_to_lds(a2, ob, 4 * kq + 2, nb);
        transpose_to_lds(a3, ob, 4 * kq + 3, nb);
    } else {
        const int kw = t & 31;
        const int64_t kwg = k0 / 8 + kw;                  // input word column
        uint32_t a[4][8];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int nb = (t >> 5) + 8 * m;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int64_t n = n0 + 8 * nb + r;
                a[m][r] = (n < N && kwg < wpr) ? (uint32_t)qweight[n * wpr + kwg] : 0u;
            }
        }
#pragma unroll
        for (int m = 0; m < 4; ++m) transpose_to_lds(a[m], ob, kw, (t >> 5) + 8 * m);
    }
    __syncthreads();
    // 256 k-rows x 32 words: 8 lanes per row, 4 words (16 B) each
    const int q = t & 7;
#pragma unroll
    for (int pass = 0; pass < 8; ++pass) {
        const int kr = (t >> 3) + 32 * pass;
        const int64_t k = k0 + kr;
        if (k >= K) continue;
        const int sw = kr >> 3;                           // the swizzle of this row (its kw)
        uint32_t w[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = ob[kr][(4 * q + e) ^ sw];
        const int64_t c0 = n0 / 8 + 4 * q;                // output word column
        int32_t* dst = qweight_t + k * wpr_t + c0;
        if (c0 + 3 < wpr_t && ((uintptr_t)dst & 15) == 0) {
            if constexpr (NT)
                __builtin_nontemporal_store(u32x4{w[0], w[1], w[2], w[3]}, (u32x4*)dst);
            else
                *(uint4*)dst = make_uint4(w[0], w[1], w[2], w[3]);
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (c0 + e < wpr_t) dst[e] = (int32_t)w[e];
        }
    }
}

// scales / qzeros (round 5): one 128-thread workgroup per 64 (n) x 32 (g) tile.  Scales: two
// rows' 16-B pieces per lane, paired into 32-bit words (n even, n + 1) and staged as
// [g][n / 2] in LDS (column XOR-swizzled by bit 3 of g: 2-way writes, the 64-lane minimum),
// stored as 128-B output row pieces.  qzeros: the 8 x 8 nibble transpose of the qweight tile
// on 32 lanes (rows 8 c .. 8 c + 7 at word gw), staged and stored as row pieces.
constexpr int kGN = 64, kGG = 32;
__device__ __forceinline__ int gswz(int g) { return 16 * ((g >> 3) & 1); }
template <bool VEC>
__global__ __launch_bounds__(128) void awq_export_group_kernel(const int32_t* __restrict__ qzeros,
                                                               const uint16_t* __restrict__ scales, int64_t N,
                                                               int64_t G, int32_t* __restrict__ qzeros_t,
                                                               uint16_t* __restrict__ scales_t) {
    __shared__ uint32_t sc[kGG][kGN / 2];                 // [g][n pair], swizzled
    __shared__ uint32_t qz[kGG][kGN / 8];                 // [g][output word column]
    const int64_t n0 = (int64_t)blockIdx.x * kGN, g0 = (int64_t)blockIdx.y * kGG;
    const int64_t wpr_z = (G + 7) / 8, wpr_t = N / 8;
    const int t = threadIdx.x;
    {
        const int p = t >> 2, gq = t & 3;                 // rows n0 + 2p, n0 + 2p + 1; g0 + 8 gq ..
        const int64_t n = n0 + 2 * p, g = g0 + 8 * gq;
        uint16_t lo[8], hi[8];
        if constexpr (VEC) {
            uint4 x = make_uint4(0, 0, 0, 0), y = x;
            if (n < N && g < G) {
                x = *(const uint4*)(scales + n * G + g);
                y = *(const uint4*)(scales + (n + 1) * G + g);
            }
            const uint32_t xs[4] = {x.x, x.y, x.z, x.w}, ys[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                lo[2 * e] = (uint16_t)xs[e]; lo[2 * e + 1] = (uint16_t)(xs[e] >> 16);
                hi[2 * e] = (uint16_t)ys[e]; hi[2 * e + 1] = (uint16_t)(ys[e] >> 16);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const bool ok = n < N && g + i < G;
                lo[i] = ok ? scales[n * G + g + i] : (uint16_t)0;
                hi[i] = ok ? scales[(n + 1) * G + g + i] : (uint16_t)0;
            }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int gr = 8 * gq + i;
            sc[gr][p ^ gswz(gr)] = (uint32_t)lo[i] | ((uint32_t)hi[i] << 16);
        }
    }
    if (t < 32) {
        const int c = t >> 2, gw = t & 3;                 // rows n0 + 8c .., zero-point word g0 / 8 + gw
        const int64_t w = g0 / 8 + gw;
        uint32_t a[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const int64_t n = n0 + 8 * c + r;
            a[r] = (n < N && w < wpr_z) ? (uint32_t)qzeros[n * wpr_z + w] : 0u;
        }
        uint32_t b[8];
        nibble_transpose8(a, b);
#pragma unroll
        for (int j = 0; j < 8; ++j) qz[8 * gw + j][c] = b[j];
    }
    __syncthreads();
    // scales_t: 32 rows x 64 n = 8 pieces of 16 B per row, 2 per lane
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        const int idx = t + 128 * m, gr = idx >> 3, q = idx & 7;
        const int64_t g = g0 + gr, n = n0 + 8 * q;
        if (g >= G || n >= N) continue;
        const uint32_t* src = &sc[gr][(4 * q) ^ gswz(gr)];
        uint16_t* dst = scales_t + g * N + n;
        if constexpr (VEC) {
            *(uint4*)dst = *(const uint4*)src;
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                dst[2 * e] = (uint16_t)src[e];
                dst[2 * e + 1] = (uint16_t)(src[e] >> 16);
            }
        }
    }
    // qzeros_t: 32 rows x 8 words, one word per lane and pass
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        const int idx = t + 128 * m, gr = idx >> 3, c = idx & 7;
        const int64_t g = g0 + gr, cw = n0 / 8 + c;
        if (g < G && cw < wpr_t) qzeros_t[g * wpr_t + cw] = (int32_t)qz[gr][c];
    }
}

}  // namespace

hipError_t launch_export_gemm(const int32_t* qweight, const int32_t* qzeros, const uint16_t* scales, int64_t N,
                              int64_t K, int64_t group_size, int32_t* qweight_t, int32_t* qzeros_t,
                              uint16_t* scales_t, hipStream_t stream) {
    if ((K + kT2 - 1) / kT2 > 65535) return hipErrorInvalidConfiguration;   // grid.y bound
    // n tiles fastest: concurrent workgroups write neighbouring pieces of the same output rows
    const dim3 grid((unsigned)((N + kT2 - 1) / kT2), (unsigned)((K + kT2 - 1) / kT2));
    const bool vec = K % 32 == 0 && ((uintptr_t)qweight & 15) == 0;
    const bool nt = N * K / 2 >= (int64_t)AWQ_EXPORT_NT_MIN;
    auto kern = vec ? (nt ? awq_export_qweight_kernel<true, true> : awq_export_qweight_kernel<true, false>)
                    : (nt ? awq_export_qweight_kernel<false, true> : awq_export_qweight_kernel<false, false>);
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, stream, qweight, N, K, qweight_t);
    if (hipError_t e = hipPeekAtLastError()) return e;
    const int64_t G = K / group_size;
    const dim3 ggrid((unsigned)((N + kGN - 1) / kGN), (unsigned)((G + kGG - 1) / kGG));
    if (G % 8 == 0 && ((uintptr_t)scales & 15) == 0 && ((uintptr_t)scales_t & 15) == 0)
        hipLaunchKernelGGL(awq_export_group_kernel<true>, ggrid, dim3(128), 0, stream, qzeros, scales, N, G, qzeros_t,
                           scales_t);
    else
        hipLaunchKernelGGL(awq_export_group_kernel<false>, ggrid, dim3(128), 0, stream, qzeros, scales, N, G, qzeros_t,
                           scales_t);
    return hipPeekAtLastError();
}

}  // namespace awq
