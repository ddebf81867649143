// dq_probe.hip — HBM ceiling of dequantize_packed's memory structure (not part of the library):
// per four fp32 outputs (one 16-B store, 1 KiB per wave instruction) 2 B of packed words read
// (4-bit: a dword shared by a lane pair) plus the row's scale / qzeros lines — a 1 : 8
// read : write stream.  Variants: store only, and the 1 : 8 mix with U quads per lane (loads
// issued first), the batched kernel's shape.  One JSON line per variant and size.
//   hipcc -O3 --offload-arch=gfx950 scripts/dq_probe.hip -o /tmp/dq_probe && /tmp/dq_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

// WR_ONLY: no loads.  Thread t of block b handles quads b * 256 U + 256 k + t, k < U.
template <int U, bool WR_ONLY, bool PLAIN = false>
__global__ __launch_bounds__(256) void dq_mix_kernel(const uint32_t* __restrict__ words, float* __restrict__ out,
                                                     int64_t quads) {
    const int64_t q0 = (int64_t)blockIdx.x * (256 * U) + threadIdx.x;
    uint32_t w[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const int64_t q = q0 + 256 * k;
        const uint32_t* a = words + min(q, quads - 1) / 2;
        w[k] = WR_ONLY ? (uint32_t)q : PLAIN ? *a : __builtin_nontemporal_load(a);
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const int64_t q = q0 + 256 * k;
        if (q >= quads) break;
        const uint32_t v = w[k] >> (16 * (int)(q & 1));
        const f4 o = {(float)(v & 15u), (float)((v >> 4) & 15u), (float)((v >> 8) & 15u), (float)((v >> 12) & 15u)};
        __builtin_nontemporal_store(o, (f4*)(out + 4 * q));
    }
}

// Persistent form: gridDim.x blocks loop over the chunks of 256 U quads, the next chunk's
// words loaded before the current chunk's stores (software pipelined), so a wave keeps
// stores and loads in flight without wave turnover.
template <int U>
__global__ __launch_bounds__(256) void dq_persist_kernel(const uint32_t* __restrict__ words, float* __restrict__ out,
                                                         int64_t quads) {
    const int64_t chunks = (quads + 256 * U - 1) / (256 * U);
    int64_t c = blockIdx.x;
    uint32_t w[U];
    auto load = [&](int64_t cc) {
#pragma unroll
        for (int k = 0; k < U; ++k) w[k] = words[min(cc * (256 * U) + 256 * k + threadIdx.x, quads - 1) / 2];
    };
    if (c < chunks) load(c);
    for (; c < chunks; c += gridDim.x) {
        uint32_t cur[U];
#pragma unroll
        for (int k = 0; k < U; ++k) cur[k] = w[k];
        if (c + gridDim.x < chunks) load(c + gridDim.x);
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int64_t q = c * (256 * U) + 256 * k + threadIdx.x;
            if (q >= quads) break;
            const uint32_t v = cur[k] >> (16 * (int)(q & 1));
            const f4 o = {(float)(v & 15u), (float)((v >> 4) & 15u), (float)((v >> 8) & 15u), (float)((v >> 12) & 15u)};
            __builtin_nontemporal_store(o, (f4*)(out + 4 * q));
        }
    }
}

template <int U>
static void run_persist(const char* name, int blocks_per_cu, const uint32_t* words, float* out, int64_t elems,
                        hipEvent_t a, hipEvent_t b) {
    const int64_t quads = elems / 4;
    const dim3 grid(256u * blocks_per_cu);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((dq_persist_kernel<U>), grid, dim3(256), 0, 0, words, out, quads);
    const int iters = 20;
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL((dq_persist_kernel<U>), grid, dim3(256), 0, 0, words, out, quads);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double us = ms * 1e3 / iters;
    printf("{\"probe\": \"%s\", \"U\": %d, \"blocks_per_cu\": %d, \"elements\": %lld, \"us\": %.1f, \"GBs\": %.1f}\n",
           name, U, blocks_per_cu, (long long)elems, us, ((double)elems * 4 + (double)elems / 2) / us / 1e3);
}

template <int U, bool WR_ONLY, bool PLAIN = false>
static void run(const char* name, const uint32_t* words, float* out, int64_t elems, hipEvent_t a, hipEvent_t b) {
    const int64_t quads = elems / 4;
    const dim3 grid((unsigned)((quads + 256 * U - 1) / (256 * U)));
    for (int i = 0; i < 3; ++i)
        hipLaunchKernelGGL((dq_mix_kernel<U, WR_ONLY, PLAIN>), grid, dim3(256), 0, 0, words, out, quads);
    const int iters = 20;
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < iters; ++i)
        hipLaunchKernelGGL((dq_mix_kernel<U, WR_ONLY, PLAIN>), grid, dim3(256), 0, 0, words, out, quads);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double us = ms * 1e3 / iters;
    const double bytes = (double)elems * 4 + (WR_ONLY ? 0.0 : (double)elems / 2);
    printf("{\"probe\": \"%s\", \"U\": %d, \"elements\": %lld, \"us\": %.1f, \"GBs\": %.1f}\n", name, U,
           (long long)elems, us, bytes / us / 1e3);
}


// WIDE: a wave's 512 quads need 1 KiB of packed words = ONE 16-B load per lane.  LDS = 1:
// the words go through a per-wave LDS slice, quad k * 64 + lane reads its word back
// (ds_read_b32) and every store instruction covers 1 KiB contiguous; LDS = 0: the lane
// converts its own 4 words (8 quads = 128 B of output, 8 stores at a 128-B lane stride).
template <bool LDS>
__global__ __launch_bounds__(256) void dq_wide_kernel(const uint32_t* __restrict__ words, float* __restrict__ out,
                                                      int64_t quads) {
    __shared__ uint32_t slice[4][256];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t q0 = ((int64_t)blockIdx.x * 4 + wid) * 512;     // the wave's first quad
    if (q0 >= quads) return;
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    const u4 w4 = __builtin_nontemporal_load((const u4*)(words + q0 / 2) + lane);
    if (LDS) {
        *(u4*)&slice[wid][4 * lane] = w4;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int qq = k * 64 + lane;
            const uint32_t v = slice[wid][qq >> 1] >> (16 * (qq & 1));
            const f4 o = {(float)(v & 15u), (float)((v >> 4) & 15u), (float)((v >> 8) & 15u), (float)((v >> 12) & 15u)};
            __builtin_nontemporal_store(o, (f4*)(out + 4 * (q0 + qq)));
        }
    } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t v = w4[k >> 1] >> (16 * (k & 1));
            const f4 o = {(float)(v & 15u), (float)((v >> 4) & 15u), (float)((v >> 8) & 15u), (float)((v >> 12) & 15u)};
            __builtin_nontemporal_store(o, (f4*)(out + 4 * (q0 + 8 * lane + k)));
        }
    }
}

template <bool LDS>
static void run_wide(const char* name, const uint32_t* words, float* out, int64_t elems, hipEvent_t a, hipEvent_t b) {
    const int64_t quads = elems / 4;
    const dim3 grid((unsigned)((quads + 2047) / 2048));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((dq_wide_kernel<LDS>), grid, dim3(256), 0, 0, words, out, quads);
    const int iters = 20;
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL((dq_wide_kernel<LDS>), grid, dim3(256), 0, 0, words, out, quads);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double us = ms * 1e3 / iters;
    printf("{\"probe\": \"%s\", \"elements\": %lld, \"us\": %.1f, \"GBs\": %.1f}\n", name, (long long)elems, us,
           ((double)elems * 4 + (double)elems / 2) / us / 1e3);
}

int main() {
    const int64_t sizes[] = {14336LL * 4096, 128256LL * 4096};
    for (int64_t elems : sizes) {
        uint32_t* words;
        float* out;
        if (hipMalloc(&words, elems / 2) != hipSuccess || hipMalloc(&out, elems * 4) != hipSuccess) return 1;
        (void)hipMemset(words, 0x5A, elems / 2);
        hipEvent_t a, b;
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&b);
        run<1, true>("store_only", words, out, elems, a, b);
        run<2, true>("store_only", words, out, elems, a, b);
        run<4, true>("store_only", words, out, elems, a, b);
        run<8, true>("store_only", words, out, elems, a, b);
        run<1, false>("read1_write8", words, out, elems, a, b);
        run<2, false>("read1_write8", words, out, elems, a, b);
        run<4, false>("read1_write8", words, out, elems, a, b);
        run<8, false>("read1_write8", words, out, elems, a, b);
        run<4, false, true>("read1_write8_plain", words, out, elems, a, b);
        run_persist<4>("persist_read1_write8", 4, words, out, elems, a, b);
        run_persist<4>("persist_read1_write8", 8, words, out, elems, a, b);
        run_persist<2>("persist_read1_write8", 8, words, out, elems, a, b);
        run_persist<8>("persist_read1_write8", 4, words, out, elems, a, b);
        run_wide<true>("wide_load_lds", words, out, elems, a, b);
        (void)hipFree(words);
        (void)hipFree(out);
    }
    return 0;
}
