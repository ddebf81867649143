// Exhaustive check of the weight-mean quotient (csrc/awq_actsearch.hip wmean_quot): for every
// pair of non-negative finite 16-bit floats x <= m (bf16 and fp16), den = fp32(m + 1e-6f),
// the Markstein form RN(q0 + e r) with r = RN(1 / den), q0 = RN(x r), e = fma(-q0, den, x)
// equals the IEEE quotient RN(x / den) bit for bit whenever the kernel's guard
// (x == 0 || x >= 2^-60) && den <= 2^60 takes it.  Exit status 0 = no mismatch.
//   gcc -O2 -mfma -fopenmp scripts/experiments/markstein_check.c -lm -o /tmp/markstein_check
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static float from_bf16(uint32_t b) {
    const uint32_t u = b << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}
static float from_f16(uint32_t h) {
    const int e = (h >> 10) & 31, m = h & 1023;
    if (e == 31) return m ? NAN : INFINITY;
    return e ? ldexpf((float)(1024 + m), e - 25) : ldexpf((float)m, -24);
}
static uint32_t bits_of(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}

static long check(int bf, long* fast_pairs) {
    long bad = 0, fast = 0;
#pragma omp parallel for reduction(+ : bad, fast) schedule(dynamic, 64)
    for (uint32_t mb = 0; mb < 0x8000; ++mb) {
        const float m = bf ? from_bf16(mb) : from_f16(mb);
        if (!isfinite(m)) continue;
        volatile float vden = m + 1e-6f;
        const float den = vden;
        volatile float vr = 1.0f / den;
        const float r = vr;
        if (!(den <= 0x1p60f)) continue;
        for (uint32_t xb = 0; xb < 0x8000; ++xb) {
            const float x = bf ? from_bf16(xb) : from_f16(xb);
            if (!isfinite(x) || x > m) continue;
            if (!(x == 0.0f || x >= 0x1p-60f)) continue;
            volatile float vq = x / den;
            const float q0 = x * r;
            const float e = fmaf(-q0, den, x);
            const float q1 = fmaf(e, r, q0);
            ++fast;
            bad += bits_of(q1) != bits_of(vq);
        }
    }
    *fast_pairs = fast;
    return bad;
}

int main(void) {
    long fast_bf, fast_h;
    const long bad_bf = check(1, &fast_bf), bad_h = check(0, &fast_h);
    printf("bf16: %ld guarded pairs, %ld mismatches\nfp16: %ld guarded pairs, %ld mismatches\n", fast_bf, bad_bf,
           fast_h, bad_h);
    return (bad_bf || bad_h) ? 1 : 0;
}
