// mix_probe.hip — HBM rate of the quantizer's memory structure (4 KiB read : 1 KiB write
// per tile) under variants of tile size per wave, cache policy, workgroup size and store
// scheduling; tuning probe, not part of the library.  Prints one JSON line per variant.
//   hipcc -O3 --offload-arch=gfx950 scripts/mix_probe.hip -o scripts/mix_probe && scripts/mix_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

// NT tiles of 4 KiB per wave; every tile's 4 loads xor-folded into one 16-B store per lane
// (1 KiB per tile).  PIPE: issue tile t+1's loads before storing tile t.  WR = 0: read only.
template <int NT, int WPB, int LPOL, int SPOL, bool PIPE, int WR>
__global__ __launch_bounds__(64 * WPB) void mix_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                       int64_t tiles) {
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t t0 = ((int64_t)blockIdx.x * WPB + wid) * NT;
    if (t0 >= tiles) return;
    const __amdgpu_buffer_rsrc_t rs = rsrc(src + t0 * 4096, 4096 * NT);
    const __amdgpu_buffer_rsrc_t rd = rsrc(dst + t0 * 1024, 1024 * NT);
    if (!PIPE) {
        u4 v[NT][4];
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                v[t][j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(t * 4096 + j * 1024 + lane * 16), 0, LPOL);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const u4 x = v[t][0] ^ v[t][1] ^ v[t][2] ^ v[t][3];
            if (WR) __builtin_amdgcn_raw_buffer_store_b128(x, rd, (uint32_t)(t * 1024 + lane * 16), 0, SPOL);
            else if (x.x == 0x12345678u && x.y == 7u) __builtin_amdgcn_raw_buffer_store_b32(x.z, rd, 0, 0, 0);
        }
    } else {
        u4 a[4], b[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(j * 1024 + lane * 16), 0, LPOL);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            if (t + 1 < NT) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    b[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)((t + 1) * 4096 + j * 1024 + lane * 16), 0,
                                                                 LPOL);
            }
            const u4 x = a[0] ^ a[1] ^ a[2] ^ a[3];
            __builtin_amdgcn_raw_buffer_store_b128(x, rd, (uint32_t)(t * 1024 + lane * 16), 0, SPOL);
#pragma unroll
            for (int j = 0; j < 4; ++j) a[j] = b[j];
        }
    }
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <int NT, int WPB, int LPOL, int SPOL, bool PIPE, int WR>
void run(const char* name, uint8_t* a, uint8_t* b, int64_t bytes) {
    const int64_t tiles = bytes / 4096;
    const int64_t per_block = (int64_t)NT * WPB;
    dim3 grid((unsigned)((tiles + per_block - 1) / per_block)), block(64 * WPB);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const double t0 = now();   // >= 150 ms of this variant before timing (clock ramp)
    while (now() - t0 < 0.15) {
        for (int w = 0; w < 4; ++w) hipLaunchKernelGGL((mix_kernel<NT, WPB, LPOL, SPOL, PIPE, WR>), grid, block, 0, 0, a, b, tiles);
        hipDeviceSynchronize();
    }
    const int iters = 20;
    hipEventRecord(e0, 0);
    for (int w = 0; w < iters; ++w) hipLaunchKernelGGL((mix_kernel<NT, WPB, LPOL, SPOL, PIPE, WR>), grid, block, 0, 0, a, b, tiles);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double moved = (WR ? 1.25 : 1.0) * (double)bytes * iters;
    printf("{\"variant\": \"%s\", \"tiles_per_wave\": %d, \"waves_per_block\": %d, \"load_pol\": %d, \"store_pol\": %d, "
           "\"pipelined\": %d, \"writes\": %d, \"us_per_launch\": %.1f, \"GBs\": %.1f}\n",
           name, NT, WPB, LPOL, SPOL, (int)PIPE, WR, ms * 1e3 / iters, moved / (ms / 1e3) / 1e9);
    fflush(stdout);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main(int argc, char** argv) {
    if (argc > 1) {   // size sweep: the ceiling structure (1 wave per workgroup) and read-only, 1..N GiB
        const int64_t max_gib = atol(argv[1]);
        uint8_t *a, *b;
        if (hipMalloc(&a, max_gib << 30) != hipSuccess || hipMalloc(&b, (max_gib << 30) / 4) != hipSuccess) return 1;
        hipMemset(a, 1, max_gib << 30);
        hipMemset(b, 0, (max_gib << 30) / 4);
        hipDeviceSynchronize();
        for (int64_t g = 1; g <= max_gib; g *= 2) {
            char name[64];
            snprintf(name, sizeof name, "size %lld GiB", (long long)g);
            run<1, 1, 2, 2, false, 1>(name, a, b, g << 30);
            run<1, 1, 2, 2, false, 0>(name, a, b, g << 30);
        }
        return 0;
    }
    const int64_t bytes = 4LL << 30;   // 4 GiB read per launch (>> the 256 MiB Infinity Cache)
    uint8_t *a, *b;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes / 4) != hipSuccess) return 1;
    hipMemset(a, 1, bytes);
    hipMemset(b, 0, bytes / 4);
    hipDeviceSynchronize();
    for (int r = 0; r < 2; ++r) {
        run<1, 1, 2, 2, false, 1>("1 wave per block", a, b, bytes);
        run<1, 2, 2, 2, false, 1>("2 waves per block", a, b, bytes);
        run<1, 8, 2, 2, false, 1>("ceiling (library structure)", a, b, bytes);
        run<1, 8, 2, 2, false, 0>("read only", a, b, bytes);
        run<1, 8, 2, 0, false, 1>("store default policy", a, b, bytes);
        run<1, 8, 2, 1, false, 1>("store sc0", a, b, bytes);
        run<1, 8, 2, 16, false, 1>("store sc1", a, b, bytes);
        run<1, 8, 2, 3, false, 1>("store sc0 nt", a, b, bytes);
        run<1, 8, 0, 2, false, 1>("load default policy", a, b, bytes);
        run<1, 8, 1, 2, false, 1>("load sc0", a, b, bytes);
        run<1, 4, 2, 2, false, 1>("4 waves per block", a, b, bytes);
        run<1, 16, 2, 2, false, 1>("16 waves per block", a, b, bytes);
        run<2, 8, 2, 2, false, 1>("2 tiles per wave", a, b, bytes);
        run<2, 4, 2, 2, false, 1>("2 tiles per wave, 4 wpb", a, b, bytes);
        run<2, 8, 2, 2, true, 1>("2 tiles pipelined", a, b, bytes);
        run<4, 8, 2, 2, true, 1>("4 tiles pipelined", a, b, bytes);
        run<4, 4, 2, 2, true, 1>("4 tiles pipelined, 4 wpb", a, b, bytes);
        run<8, 4, 2, 2, true, 1>("8 tiles pipelined, 4 wpb", a, b, bytes);
    }
    hipFree(a);
    hipFree(b);
    return 0;
}
