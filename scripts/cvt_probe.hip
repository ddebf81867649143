// cvt_probe.hip — rounding and saturation of v_cvt_pk_u8_f32 on gfx950 (not part of the
// library): whether one conversion can replace rint + clamp(0, 255) in the quantizers' pack.
//   hipcc -O2 --offload-arch=gfx950 scripts/cvt_probe.hip -o /tmp/cvt_probe && /tmp/cvt_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

__global__ void cvt_kernel(const float* in, uint32_t* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = __builtin_amdgcn_cvt_pk_u8_f32(in[i], 0, 0u);
}

int main() {
    const float vals[] = {0.0f, -0.0f, 0.25f, 0.5f, 0.75f, 1.5f, 2.5f, 3.5f, 4.5f, 0.49999997f, 0.50000006f,
                          -0.5f, -0.50000006f, -0.7f, -1.0f, -300.0f, 7.5f, 8.5f, 15.5f, 16.49f, 254.5f, 255.4f,
                          255.5f, 256.0f, 300.0f, 1e10f, INFINITY, -INFINITY, NAN, 127.5f, 128.5f};
    const int n = sizeof(vals) / sizeof(vals[0]);
    float* d_in;
    uint32_t* d_out;
    uint32_t out[64];
    if (hipMalloc(&d_in, sizeof(vals)) != hipSuccess || hipMalloc(&d_out, n * 4) != hipSuccess) return 1;
    if (hipMemcpy(d_in, vals, sizeof(vals), hipMemcpyHostToDevice) != hipSuccess) return 1;
    hipLaunchKernelGGL(cvt_kernel, dim3(1), dim3(64), 0, 0, d_in, d_out, n);
    if (hipMemcpy(out, d_out, n * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    int rne_sat_ok = 1;
    for (int i = 0; i < n; ++i) {
        const float v = vals[i];
        // expected under "round to nearest even, then saturate to [0, 255], NaN -> 0"
        float e = std::isnan(v) ? 0.0f : std::nearbyint(v);
        e = e < 0.0f ? 0.0f : (e > 255.0f ? 255.0f : e);
        const uint32_t exp = (uint32_t)e;
        const uint32_t got = out[i] & 0xFFu;
        if (got != exp) rne_sat_ok = 0;
        printf("{\"in\": \"%a\", \"value\": %.9g, \"byte\": %u, \"rne_saturate\": %u}\n", v, v, got, exp);
    }
    printf("{\"cvt_pk_u8_f32_is_rne_saturate\": %s}\n", rne_sat_ok ? "true" : "false");
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    return 0;
}
