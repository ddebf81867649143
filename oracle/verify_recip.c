/* verify_recip.c — exhaustive check of the identity the bf16 HIP fast path relies on
 * (TEST INFRASTRUCTURE ONLY):
 *
 *   for every finite bf16 x and every finite bf16 s >= RN_bf16(1e-10):
 *       RN_bf16( x * RN_f32(1/s) ) == RN_bf16( RN_f32(x / s) )
 *
 * i.e. one correctly rounded reciprocal per group + one fp32 multiply per element
 * reproduces awq.py:245's `tensor / scale` (torch bf16 divide = fp32 divide + RNE)
 * and awq.py:210's `t_min / scale` bit for bit.  Also reports the fp16 analogue
 * (expected to FAIL, which is why fp16 inputs use a true division).
 * Usage: verify_recip [bf16|f16|f16m|f16s|f16f|chain16|f16scale|alpha] -> prints mismatches, exit 0 iff none (bf16;
 * f16m: the fp16 Markstein-corrected quotient; f16s: the fp16 plain product for s < 14;
 * f16f: the same product rounded once, straight to fp16; chain16: the search's packed-fp16 rint
 * and clamp; alpha: the search's candidate factor). */
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include "awq_oracle.h"

static int finite16(uint16_t h, int bf) {
    return bf ? ((h & 0x7F80u) != 0x7F80u) : ((h & 0x7C00u) != 0x7C00u);
}
static float dec(uint16_t h, int bf) { return bf ? oracle_bf16_to_f32(h) : oracle_f16_to_f32(h); }
static uint16_t enc(float f, int bf) { return bf ? oracle_f32_to_bf16(f) : oracle_f32_to_f16(f); }

/* fp16 fast path (csrc/awq_fast.hip, Fmt<F16>::div): r = RN_f32(1/s), q0 = RN_f32(x*r),
 * e = fma(-s, q0, x) (exact residual), q1 = fma(e, r, q0) — must give RN_f16(x / s) for
 * every finite fp16 x and every positive finite fp16 s (scale clamp min RN_f16(1e-10) = 0,
 * s = 0 takes the IEEE-division special path).  Zeros compare by value (-0 == +0: the
 * quantized integer does not depend on the sign of a zero quotient). */
static int check_f16_markstein(void) {
    long long mismatches = 0, pairs = 0;
#pragma omp parallel for reduction(+ : mismatches, pairs) schedule(dynamic, 64)
    for (int si = 1; si < 0x7C00; ++si) {
        float s = oracle_f16_to_f32((uint16_t)si);
        volatile float one = 1.0f;
        float r = one / s;
        for (int xi = 0; xi < 65536; ++xi) {
            uint16_t xh = (uint16_t)xi;
            if ((xh & 0x7C00u) == 0x7C00u) continue;
            float x = oracle_f16_to_f32(xh);
            float q0 = x * r;
            float e = fmaf(-s, q0, x);
            float q1 = fmaf(e, r, q0);
            float a = oracle_f16_to_f32(oracle_f32_to_f16(q1)), b = oracle_f16_to_f32(oracle_f32_to_f16(x / s));
            pairs++;
            if (!(a == b)) mismatches++;
        }
    }
    printf("f16 markstein: pairs=%lld mismatches=%lld\n", pairs, mismatches);
    return mismatches == 0 ? 0 : 1;
}

/* fp16 plain product for small scales (csrc/awq_fast.hip FmtF16::quot_plain): for every
 * finite fp16 x and every positive fp16 s < 14, RN_f16(RN_f32(x * RN_f32(1/s))) equals
 * RN_f16(x / s).  Also reports the smallest scale for which the plain product fails. */
static int check_f16_small(void) {
    long long mismatches = 0, pairs = 0;
    int first_bad = 0x7C00;
#pragma omp parallel for reduction(+ : mismatches, pairs) reduction(min : first_bad) schedule(dynamic, 64)
    for (int si = 1; si < 0x7C00; ++si) {
        float s = oracle_f16_to_f32((uint16_t)si);
        volatile float one = 1.0f;
        float r = one / s;
        for (int xi = 0; xi < 65536; ++xi) {
            uint16_t xh = (uint16_t)xi;
            if ((xh & 0x7C00u) == 0x7C00u) continue;
            float x = oracle_f16_to_f32(xh);
            float a = oracle_f16_to_f32(oracle_f32_to_f16(x * r)), b = oracle_f16_to_f32(oracle_f32_to_f16(x / s));
            if (s < 14.0f) pairs++;
            if (!(a == b)) {
                if (s < 14.0f) mismatches++;
                if (si < first_bad) first_bad = si;
            }
        }
    }
    printf("f16 small-scale plain product: pairs=%lld mismatches=%lld first_failing_scale=%g\n", pairs,
           mismatches, oracle_f16_to_f32((uint16_t)first_bad));
    return mismatches == 0 ? 0 : 1;
}

/* RN_f16 of a double (round to nearest even, fp16 subnormals, overflow to inf): the quantum of
 * |d|'s binade (or the subnormal quantum 2^-24), nearbyint in the default RNE mode. */
static double rn_f16_of_double(double d) {
    if (d == 0.0 || d != d) return d;
    const double a = fabs(d);
    int e;
    frexp(a, &e);                         /* a in [2^(e-1), 2^e) */
    const int ex = (e - 1 < -14) ? -14 : e - 1;
    const double q = ldexp(1.0, ex - 10);
    double r = nearbyint(a / q) * q;
    if (r >= 65520.0) r = INFINITY;       /* (65504 + 16: the RNE overflow threshold) */
    else if (r > 65504.0) r = 65504.0;
    return d < 0 ? -r : r;
}

/* The clip search's fp16 chain (csrc/awq_fast.hip chunk_err_f16p) forms t = RN_f16(x * r) with
 * ONE rounding (v_fma_mixlo_f16 / v_fma_mixhi_f16: the exact product rounded to fp16): for every
 * finite fp16 x and every positive fp16 s < 14 it must equal RN_f16(RN_f32(x / s)) (torch's fp16
 * division), by value. */
static int check_f16_fused(void) {
    long long mismatches = 0, pairs = 0;
#pragma omp parallel for reduction(+ : mismatches, pairs) schedule(dynamic, 64)
    for (int si = 1; si < 0x7C00; ++si) {
        const float s = oracle_f16_to_f32((uint16_t)si);
        if (!(s < 14.0f)) continue;
        volatile float one = 1.0f;
        const float r = one / s;
        for (int xi = 0; xi < 65536; ++xi) {
            const uint16_t xh = (uint16_t)xi;
            if ((xh & 0x7C00u) == 0x7C00u) continue;
            const float x = oracle_f16_to_f32(xh);
            const double a = rn_f16_of_double((double)x * (double)r);   /* exact product, one rounding */
            const float b = oracle_f16_to_f32(oracle_f32_to_f16(x / s));
            pairs++;
            if (!(a == (double)b)) mismatches++;
        }
    }
    printf("f16 fused small-scale product: pairs=%lld mismatches=%lld\n", pairs, mismatches);
    return mismatches == 0 ? 0 : 1;
}

/* The clip search's packed-fp16 integer steps (csrc/awq_fast.hip chunk_err_f16p, chunk_err_bf16h):
 * q = clamp(rint(u), qmin, qmax) formed as min(max(RN_f16(h + OFF), 1024), 1024 + qmax - qmin)
 * - OFF + ... with OFF = 1024 - qmin, h = u for an fp16 u and h = RN_f16(u) for a bf16 u (f32
 * form).  Every finite / infinite fp16 and bf16 u, 4 / 8 bit, asymmetric / symmetric. */
static int check_chain16(void) {
    long long cases = 0, mismatches = 0;
    for (int bits = 4; bits <= 8; bits += 4)
        for (int sym = 0; sym <= 1; ++sym) {
            const double qmin = sym ? -(double)(1 << (bits - 1)) : 0.0;
            const double qmax = sym ? (double)((1 << (bits - 1)) - 1) : (double)((1 << bits) - 1);
            const double off = 1024.0 - qmin;
            for (int bf = 0; bf <= 1; ++bf)
                for (int i = 0; i < 65536; ++i) {
                    const uint16_t hb = (uint16_t)i;
                    const float u = dec(hb, bf);
                    if (u != u) continue;
                    const double h = bf ? (double)oracle_f16_to_f32(oracle_f32_to_f16(u)) : (double)u;
                    double v = rn_f16_of_double(h + off);
                    v = v < 1024.0 ? 1024.0 : v;
                    v = v > 1024.0 + qmax - qmin ? 1024.0 + qmax - qmin : v;
                    const double got = v - off;
                    double want = nearbyint((double)u);
                    want = want < qmin ? qmin : (want > qmax ? qmax : want);
                    cases++;
                    if (got != want) mismatches++;
                }
        }
    printf("packed fp16 rint + clamp: cases=%lld mismatches=%lld\n", cases, mismatches);
    return mismatches == 0 ? 0 : 1;
}

/* fp16 scale without the IEEE division (csrc/awq_quant.h FmtF16::scale, act HwFmt<F16>::scale):
 * RN_f16(d / qr) == RN_f16(d * RN_f32(1 / qr)) for every non-negative fp16 d (inf included) and
 * qr = 2^bits - 1, bits 2..8 — the group scale awq.py:202 forms from RN_f16(max - min). */
static int check_f16_scale(void) {
    long long cases = 0, mismatches = 0;
    for (int bits = 2; bits <= 8; ++bits) {
        volatile float one = 1.0f;
        const float qr = (float)((1 << bits) - 1), rq = one / qr;
        for (int h = 0; h <= 0x7C00; ++h) {
            const float d = oracle_f16_to_f32((uint16_t)h);
            const uint16_t a = oracle_f32_to_f16(d * rq), b = oracle_f32_to_f16(d / qr);
            cases++;
            if (a != b) mismatches++;
        }
    }
    printf("f16 scale d * RN(1/qr): cases=%lld mismatches=%lld\n", cases, mismatches);
    return mismatches == 0 ? 0 : 1;
}

/* The clip search's candidate factor alpha_i = RN_f32((n - i) / n) (include/awq_hip.h
 * awq_quantize_search) as the streaming kernel forms it without a division per candidate:
 * q = a * RN(1/n), r = fma(-n, q, a), alpha = fma(r, RN(1/n), q) with a = n - i — equal to the
 * IEEE quotient for every n <= 65536 and 0 <= i < n (2.1e9 pairs). */
static int check_alpha(void) {
    long long pairs = 0, mismatches = 0;
#pragma omp parallel for reduction(+ : pairs, mismatches) schedule(dynamic, 256)
    for (int n = 1; n <= 65536; ++n) {
        volatile float one = 1.0f;
        const float nf = (float)n, rn = one / nf;
        for (int i = 0; i < n; ++i) {
            const float a = (float)(n - i);
            const float q = a * rn;
            const float r = fmaf(-nf, q, a);
            const float al = fmaf(r, rn, q);
            volatile float want = a / nf;
            pairs++;
            if (memcmp(&al, (const void*)&want, 4) != 0) mismatches++;
        }
    }
    printf("alpha (n - i) / n, n <= 65536: pairs=%lld mismatches=%lld\n", pairs, mismatches);
    return mismatches == 0 ? 0 : 1;
}

int main(int argc, char** argv) {
    if (argc > 1 && strcmp(argv[1], "alpha") == 0) return check_alpha();
    if (argc > 1 && strcmp(argv[1], "f16m") == 0) return check_f16_markstein();
    if (argc > 1 && strcmp(argv[1], "f16s") == 0) return check_f16_small();
    if (argc > 1 && strcmp(argv[1], "f16f") == 0) return check_f16_fused();
    if (argc > 1 && strcmp(argv[1], "chain16") == 0) return check_chain16();
    if (argc > 1 && strcmp(argv[1], "f16scale") == 0) return check_f16_scale();
    int bf = !(argc > 1 && strcmp(argv[1], "f16") == 0);
    float lo = dec(enc(1e-10f, bf), bf);
    long long mismatches = 0, pairs = 0;
#pragma omp parallel for reduction(+ : mismatches, pairs) schedule(dynamic, 64)
    for (int si = 0; si < 65536; ++si) {
        uint16_t sh = (uint16_t)si;
        if (!finite16(sh, bf)) continue;
        float s = dec(sh, bf);
        if (!(s >= lo) || s <= 0.0f) continue;
        volatile float one = 1.0f;
        float r = one / s;
        for (int xi = 0; xi < 65536; ++xi) {
            uint16_t xh = (uint16_t)xi;
            if (!finite16(xh, bf)) continue;
            float x = dec(xh, bf);
            uint16_t a = enc(x * r, bf), b = enc(x / s, bf);
            pairs++;
            if (a != b) mismatches++;
        }
    }
    printf("%s: pairs=%lld mismatches=%lld\n", bf ? "bf16" : "f16", pairs, mismatches);
    return (bf && mismatches == 0) ? 0 : 1;
}
