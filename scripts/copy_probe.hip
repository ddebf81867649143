// copy_probe.hip — HBM copy rate vs bytes in flight per wave (tuning probe for the
// quantizer's tile size; not part of the library).
//   hipcc -O3 --offload-arch=gfx950 scripts/copy_probe.hip -o scripts/copy_probe && scripts/copy_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

// one wave copies NL KiB: NL x 16-B loads per lane, all in flight, then NL stores
template <int NL, int WPB>
__global__ __launch_bounds__(64 * WPB) void copy_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                        int64_t bytes) {
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t base = ((int64_t)blockIdx.x * WPB + wid) * (1024 * NL);
    if (base >= bytes) return;
    const uint32_t n = (uint32_t)min((int64_t)(1024 * NL), bytes - base);
    const __amdgpu_buffer_rsrc_t rs = rsrc(src + base, n), rd = rsrc(dst + base, n);
    u4 v[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) v[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(j * 1024 + lane * 16), 0, 2);
#pragma unroll
    for (int j = 0; j < NL; ++j) __builtin_amdgcn_raw_buffer_store_b128(v[j], rd, (uint32_t)(j * 1024 + lane * 16), 0, 2);
}

// read-only: NL KiB per wave, xor-reduced, one dword stored per wave
template <int NL, int WPB>
__global__ __launch_bounds__(64 * WPB) void read_kernel(const uint8_t* __restrict__ src, uint32_t* __restrict__ sink,
                                                        int64_t bytes) {
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t base = ((int64_t)blockIdx.x * WPB + wid) * (1024 * NL);
    if (base >= bytes) return;
    const __amdgpu_buffer_rsrc_t rs = rsrc(src + base, 1024 * NL);
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
        u4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(j * 1024 + lane * 16), 0, 2);
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (x == 0x12345678u) sink[lane] = x;
}

template <int NL, int WPB>
void run(const char* name, uint8_t* a, uint8_t* b, uint32_t* sink, int64_t bytes, bool rd) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int64_t per_block = 1024LL * NL * WPB;
    dim3 grid((unsigned)((bytes + per_block - 1) / per_block)), block(64 * WPB);
    for (int w = 0; w < 3; ++w) {
        if (rd) hipLaunchKernelGGL((read_kernel<NL, WPB>), grid, block, 0, 0, a, sink, bytes);
        else hipLaunchKernelGGL((copy_kernel<NL, WPB>), grid, block, 0, 0, a, b, bytes);
    }
    const int iters = 10;
    hipEventRecord(e0, 0);
    for (int w = 0; w < iters; ++w) {
        if (rd) hipLaunchKernelGGL((read_kernel<NL, WPB>), grid, block, 0, 0, a, sink, bytes);
        else hipLaunchKernelGGL((copy_kernel<NL, WPB>), grid, block, 0, 0, a, b, bytes);
    }
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double moved = (rd ? 1.0 : 2.0) * (double)bytes * iters;
    printf("{\"kernel\": \"%s\", \"KiB_per_wave\": %d, \"waves_per_block\": %d, \"GBs\": %.1f}\n", name, NL, WPB,
           moved / (ms / 1e3) / 1e9);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main() {
    const int64_t bytes = 1LL << 31;   // 2 GiB each way
    uint8_t *a, *b;
    uint32_t* sink;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess || hipMalloc(&sink, 256) != hipSuccess)
        return 1;
    hipMemset(a, 1, bytes);
    hipMemset(b, 0, bytes);
    hipDeviceSynchronize();
    for (int r = 0; r < 2; ++r) {
        run<4, 8>("copy", a, b, sink, bytes, false);
        run<8, 8>("copy", a, b, sink, bytes, false);
        run<16, 8>("copy", a, b, sink, bytes, false);
        run<4, 4>("copy", a, b, sink, bytes, false);
        run<8, 4>("copy", a, b, sink, bytes, false);
        run<4, 8>("read", a, b, sink, bytes, true);
        run<8, 8>("read", a, b, sink, bytes, true);
        run<16, 8>("read", a, b, sink, bytes, true);
    }
    hipFree(a);
    hipFree(b);
    hipFree(sink);
    return 0;
}
