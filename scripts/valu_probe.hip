// valu_probe.hip — VALU issue rate of gfx950 per instruction class, to price the VALU roofline
// of the grid-search kernels (bench.py --mode search / act).  Every wave runs ITER blocks of
// 32 instructions of one class over 8 independent registers (no dependent chains), at 2 and
// 8 waves per SIMD; reported: lane-instructions per second and cycles per instruction
// per SIMD at the clock given by --ghz (the kernel's measured GRBM clock in bench PMC runs
// is 2.39).  Tuning probe, not part of the library; only vector ALU instructions in asm.
//   hipcc -O3 --offload-arch=gfx950 scripts/valu_probe.hip -o scripts/valu_probe && scripts/valu_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int OP>
__device__ __forceinline__ void block(float (&a)[8], f2 (&p)[8], float b, float c) {
#pragma unroll
    for (int rep = 0; rep < 4; ++rep) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if constexpr (OP == 0) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[k]) : "v"(b), "v"(c));
            if constexpr (OP == 1) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p[k]) : "v"(p[(k + 1) & 7]), "v"(p[(k + 2) & 7]));
            if constexpr (OP == 2) asm volatile("v_add_f32 %0, %1, %0" : "+v"(a[k]) : "v"(b));
            if constexpr (OP == 3) asm volatile("v_cvt_pk_bf16_f32 %0, 0, %0" : "+v"(a[k]));
            if constexpr (OP == 4) asm volatile("v_rndne_f32 %0, %0" : "+v"(a[k]));
            if constexpr (OP == 5) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(b), "v"(c));
            if constexpr (OP == 6) asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(a[k]) : "v"(a[(k + 4) & 7]));
            if constexpr (OP == 7) asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(a[k]) : "v"(b), "v"(c));
            if constexpr (OP == 8) asm volatile("v_exp_f32 %0, %0" : "+v"(a[k]));
            if constexpr (OP == 9) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p[k]) : "v"(p[(k + 3) & 7]));
            if constexpr (OP == 10) asm volatile("v_cvt_f32_f16 %0, %0" : "+v"(a[k]));
            if constexpr (OP == 11) asm volatile("v_mul_f16 %0, %0, %1" : "+v"(a[k]) : "v"(b));
            if constexpr (OP == 12) asm volatile("v_max_f32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
            if constexpr (OP == 13) asm volatile("v_sub_f32 %0, %1, %0" : "+v"(a[k]) : "v"(b));
            if constexpr (OP == 14) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[k]) : "v"(b) : "vcc");
            if constexpr (OP == 15) asm volatile("v_cmp_lt_f32 vcc, %0, %1" : : "v"(a[k]), "v"(b) : "vcc");
            if constexpr (OP == 16) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p[k]) : "v"(p[(k + 3) & 7]));
            if constexpr (OP == 17) asm volatile("v_cvt_pk_f16_f32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
            if constexpr (OP == 18) asm volatile("v_pk_mul_f16 %0, %0, %1" : "+v"(a[k]) : "v"(b));
            if constexpr (OP == 19) asm volatile("v_cvt_f16_f32 %0, %0" : "+v"(a[k]));
            if constexpr (OP == 20) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
            if constexpr (OP == 21) asm volatile("v_lshlrev_b32 %0, 16, %0" : "+v"(a[k]));
            if constexpr (OP == 22) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(b), "v"(c));
            if constexpr (OP == 23) asm volatile("v_bfe_u32 %0, %0, 16, 1" : "+v"(a[k]));
            if constexpr (OP == 24) asm volatile("v_mov_b32 %0, %1" : "=v"(a[k]) : "v"(a[(k + 4) & 7]));
            if constexpr (OP == 25) asm volatile("v_add_f32_dpp %0, %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(a[k]) : "v"(a[(k + 4) & 7]));
            if constexpr (OP == 26) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
            if constexpr (OP == 27) asm volatile("v_rcp_f32 %0, %0" : "+v"(a[k]));
            if constexpr (OP == 28) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
            if constexpr (OP == 29) asm volatile("v_min_f32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
            if constexpr (OP == 30) asm volatile("v_max_i32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
            if constexpr (OP == 31) asm volatile("v_max_u32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
            if constexpr (OP == 32) asm volatile("v_min_i32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
            if constexpr (OP == 33) asm volatile("v_or_b32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
            if constexpr (OP == 34) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
            if constexpr (OP == 35) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
            if constexpr (OP == 36) asm volatile("v_add_f16 %0, %0, %1" : "+v"(a[k]) : "v"(b));
            if constexpr (OP == 37) asm volatile("v_fma_f16 %0, %0, %1, %2" : "+v"(a[k]) : "v"(b), "v"(c));
            if constexpr (OP == 38) asm volatile("v_pk_add_f16 %0, %0, %1" : "+v"(a[k]) : "v"(b));
            if constexpr (OP == 39) asm volatile("v_max_f16 %0, %0, %1" : "+v"(a[k]) : "v"(b));
            if constexpr (OP == 40) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(b), "v"(c));
            if constexpr (OP == 41) asm volatile("v_lshlrev_b32_e32 %0, %1, %0" : "+v"(a[k]) : "v"(b));
            if constexpr (OP == 42) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a[k]) : "v"(b), "v"(c));
            if constexpr (OP == 43) asm volatile("v_sub_f16 %0, %0, %1" : "+v"(a[k]) : "v"(b));
            if constexpr (OP == 44) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(a[k]));
            if constexpr (OP == 45) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[k]) : "v"(b));
            if constexpr (OP == 46) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(b), "v"(c));
            if constexpr (OP == 47) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a[k]) : "v"(b) : "vcc");
        }
    }
}

template <int OP>
__global__ __launch_bounds__(256) void probe(float* out, int iters, float b, float c) {
    float a[8];
    f2 p[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        a[k] = (float)(threadIdx.x + k);
        p[k] = f2{a[k], a[k] + 1.0f};
    }
    for (int it = 0; it < iters; ++it) block<OP>(a, p, b, c);
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += a[k] + p[k].x + p[k].y;
    out[(size_t)blockIdx.x * 256 + threadIdx.x] = s;   // vector store: keeps the work live
}

static const char* kNames[] = {"v_fma_f32",  "v_pk_fma_f32", "v_add_f32",    "v_cvt_pk_bf16_f32",
                               "v_rndne_f32", "v_med3_f32",  "v_mov_b32_dpp", "v_fma_mix_f32",
                               "v_exp_f32",   "v_pk_mul_f32", "v_cvt_f32_f16", "v_mul_f16",
                               "v_max_f32",   "v_sub_f32",   "v_cndmask_b32", "v_cmp_lt_f32",
                               "v_pk_add_f32", "v_cvt_pk_f16_f32", "v_pk_mul_f16", "v_cvt_f16_f32",
                               "v_and_b32",   "v_lshlrev_b32", "v_add3_u32",  "v_bfe_u32",
                               "v_mov_b32",   "v_add_f32_dpp", "v_mul_f32",   "v_rcp_f32",
                               "v_add_u32",   "v_min_f32",   "v_max_i32",   "v_max_u32",
                               "v_min_i32",   "v_or_b32",    "v_xor_b32",   "v_sub_u32",
                               "v_add_f16",   "v_fma_f16",   "v_pk_add_f16", "v_max_f16",
                               "v_perm_b32",  "v_lshlrev_b32_e32", "v_fmac_f32", "v_sub_f16",
                               "v_cvt_f32_u32", "v_mul_u32_u24", "v_max3_f32", "v_add_co_u32"};

template <int OP>
static void run(float* out, int cus, double ghz) {
    const int iters = 8000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int wps : {2, 8}) {
        const int blocks = cus * wps;   // 256 threads = one wave per SIMD per workgroup
        hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), 0, 0, out, 50, 1.0f, 0.5f);
        hipEventRecord(e0);
        hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0f, 0.5f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double insts_per_wave = (double)iters * 32;
        const double waves = (double)blocks * 4;
        const double lane_instr_per_s = insts_per_wave * waves * 64 / (ms * 1e-3);
        const double cyc = (ms * 1e-3) * ghz * 1e9 / (insts_per_wave * wps);   // per instruction per SIMD
        printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"T_lane_instr_per_s\": %.2f, "
               "\"cycles_per_instr_per_simd\": %.3f}\n",
               kNames[OP], wps, ms, lane_instr_per_s / 1e12, cyc);
    }
}

int main(int argc, char** argv) {
    double ghz = 2.4;
    for (int i = 1; i + 1 < argc; ++i)
        if (!strcmp(argv[i], "--ghz")) ghz = atof(argv[i + 1]);
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    float* out = nullptr;
    if (hipMalloc(&out, (size_t)cus * 8 * 256 * sizeof(float)) != hipSuccess) return 1;
    printf("{\"device\": \"%s\", \"cus\": %d, \"clock_mhz\": %d}\n", prop.gcnArchName, cus, prop.clockRate / 1000);
    run<0>(out, cus, ghz);
    run<1>(out, cus, ghz);
    run<2>(out, cus, ghz);
    run<3>(out, cus, ghz);
    run<4>(out, cus, ghz);
    run<5>(out, cus, ghz);
    run<6>(out, cus, ghz);
    run<7>(out, cus, ghz);
    run<8>(out, cus, ghz);
    run<9>(out, cus, ghz);
    run<10>(out, cus, ghz);
    run<11>(out, cus, ghz);
    run<12>(out, cus, ghz);
    run<13>(out, cus, ghz);
    run<14>(out, cus, ghz);
    run<15>(out, cus, ghz);
    run<16>(out, cus, ghz);
    run<17>(out, cus, ghz);
    run<18>(out, cus, ghz);
    run<19>(out, cus, ghz);
    run<20>(out, cus, ghz);
    run<21>(out, cus, ghz);
    run<22>(out, cus, ghz);
    run<23>(out, cus, ghz);
    run<24>(out, cus, ghz);
    run<25>(out, cus, ghz);
    run<26>(out, cus, ghz);
    run<27>(out, cus, ghz);
    run<28>(out, cus, ghz);
    run<29>(out, cus, ghz);
    run<30>(out, cus, ghz);
    run<31>(out, cus, ghz);
    run<32>(out, cus, ghz);
    run<33>(out, cus, ghz);
    run<34>(out, cus, ghz);
    run<35>(out, cus, ghz);
    run<36>(out, cus, ghz);
    run<37>(out, cus, ghz);
    run<38>(out, cus, ghz);
    run<39>(out, cus, ghz);
    run<40>(out, cus, ghz);
    run<41>(out, cus, ghz);
    run<42>(out, cus, ghz);
    run<43>(out, cus, ghz);
    run<44>(out, cus, ghz);
    run<45>(out, cus, ghz);
    run<46>(out, cus, ghz);
    run<47>(out, cus, ghz);
    hipFree(out);
    return 0;
}
