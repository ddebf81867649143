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
// qweight: one workgroup transposes a 64 (n) x 128 (k) nibble tile through LDS (reads
// 64 rows x 64 B, writes 128 rows x 32 B); scales / qzeros: one thread per output
// qzeros word, gathering 8 zero points and moving 8 scales.  HBM-bound, 1 B/element.
#include "awq_internal.h"

namespace awq {
namespace {

constexpr int kOrder[8] = {0, 2, 4, 6, 1, 3, 5, 7};
constexpr int kTileN = 64, kTileK = 128;

__global__ __launch_bounds__(256) void awq_export_qweight_kernel(const int32_t* __restrict__ qweight, int64_t N,
                                                                 int64_t K, int32_t* __restrict__ qweight_t) {
    __shared__ uint8_t nib[kTileN][kTileK + 4];   // +4: spread the column reads over banks
    const int64_t n0 = (int64_t)blockIdx.y * kTileN, k0 = (int64_t)blockIdx.x * kTileK;
    const int64_t wpr = K / 8, wpr_t = N / 8;
    const int tid = threadIdx.x;
    // load: 64 rows x 16 words, word (n, w) holds k = k0 + 8w .. +7
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const int idx = tid + 256 * m;
        const int n = idx >> 4, w = idx & 15;
        uint32_t v = 0;
        if (n0 + n < N && k0 + 8 * w < K) v = (uint32_t)qweight[(n0 + n) * wpr + k0 / 8 + w];
#pragma unroll
        for (int j = 0; j < 8; ++j) nib[n][8 * w + j] = (uint8_t)((v >> (4 * j)) & 0xFu);
    }
    __syncthreads();
    // store: 128 k-rows x 8 words, word (k, c) = columns n0 + 8c + kOrder[i] at nibble i
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const int idx = tid + 256 * m;
        const int k = idx >> 3, c = idx & 7;
        uint32_t v = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) v |= (uint32_t)nib[8 * c + kOrder[i]][k] << (4 * i);
        if (k0 + k < K && n0 + 8 * c < N) qweight_t[(k0 + k) * wpr_t + n0 / 8 + c] = (int32_t)v;
    }
}

__global__ __launch_bounds__(256) void awq_export_group_kernel(const int32_t* __restrict__ qzeros,
                                                               const uint16_t* __restrict__ scales, int64_t N,
                                                               int64_t G, int32_t* __restrict__ qzeros_t,
                                                               uint16_t* __restrict__ scales_t) {
    const int64_t wpr_z = (G + 7) / 8, wpr_t = N / 8;
    const int64_t total = G * wpr_t;
    for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < total;
         o += (int64_t)gridDim.x * blockDim.x) {
        const int64_t g = o / wpr_t, c = o - g * wpr_t;
        uint32_t v = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int64_t n = 8 * c + kOrder[i];
            const uint32_t zw = (uint32_t)qzeros[n * wpr_z + g / 8];
            v |= ((zw >> (4 * (g % 8))) & 0xFu) << (4 * i);
        }
        qzeros_t[o] = (int32_t)v;
#pragma unroll
        for (int i = 0; i < 8; ++i) scales_t[g * N + 8 * c + i] = scales[(8 * c + i) * G + g];
    }
}

}  // namespace

hipError_t launch_export_gemm(const int32_t* qweight, const int32_t* qzeros, const uint16_t* scales, int64_t N,
                              int64_t K, int64_t group_size, int32_t* qweight_t, int32_t* qzeros_t,
                              uint16_t* scales_t, hipStream_t stream) {
    const dim3 grid((unsigned)((K + kTileK - 1) / kTileK), (unsigned)((N + kTileN - 1) / kTileN));
    hipLaunchKernelGGL(awq_export_qweight_kernel, grid, dim3(256), 0, stream, qweight, N, K, qweight_t);
    if (hipError_t e = hipPeekAtLastError()) return e;
    const int64_t G = K / group_size;
    const int64_t work = G * (N / 8);
    int64_t blocks = (work + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(awq_export_group_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, qzeros, scales, N, G,
                       qzeros_t, scales_t);
    return hipPeekAtLastError();
}

}  // namespace awq
