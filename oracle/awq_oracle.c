/*
 * awq_oracle.c — CPU restatement of the reference's group quantizer.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the *checker* the parity tests,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg compare the HIP path
 * against.  Nothing in the product (awq-converter_amd/) links, loads or calls
 * it; the product has no CPU fallback.
 *
 * Pinned against tests/golden/ (outputs of the reference awq.py imported in
 * the build container by tests/golden/make_golden.py); see
 * tests/test_oracle_golden.py.
 *
 * What it restates (reference = shanefitch/AWQ-Converter, src/awq_quantizer):
 *   quantization/awq.py:173-213  _compute_scale_zp_for_group  (min/max, sym
 *                                 abs-max, scale, clamp 1e-10, zero point)
 *   quantization/awq.py:215-250  _quantize_tensor  (round(x/s + z), clamp)
 *   quantization/awq.py:286-374  _quantize_per_group (rows = dim 0, rest
 *                                 flattened, tail group zero-padded)
 *   quantization/awq.py:130-171  _calculate_scale_zp (numel < group_size:
 *                                 whole tensor or whole rows, no padding)
 *   quantization/awq.py:409-412  result dtypes (int32 / fp16 / int32), incl. the
 *                                 bits of NaN scales (oracle_nan_scale_f16)
 *   quantization/awq.py:459-539  dequantize ((q - z) * fp16 scale -> fp16)
 *
 * Arithmetic model (torch CPU eager semantics for one element-wise op on a
 * reduced-precision dtype D): compute in fp32 (fp64 for D = fp64), round the
 * result to D with round-to-nearest-even after EVERY op.  torch.round is
 * round-half-even; min/max/clamp propagate NaN; float->int32 of NaN gives
 * INT_MIN (x86 cvtt*).  fp64 scales are stored through an fp32 tensor
 * (awq.py:327) before .to(float16), i.e. RN_f16(RN_f32(s)).
 *
 * Build: make -C oracle   (gcc, no fast-math, -ffp-contract=off)
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#include "awq_oracle.h"

/* ---------------- rounding helpers ---------------- */

static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* fp32 -> bf16 bits, round-to-nearest-even (c10::BFloat16 semantics; NaN -> 0x7FC0) */
uint16_t oracle_f32_to_bf16(float f) {
    if (isnan(f)) return 0x7FC0;
    uint32_t u = f2u(f);
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}
float oracle_bf16_to_f32(uint16_t h) { return u2f((uint32_t)h << 16); }

/* fp32 -> fp16 bits, round-to-nearest-even, subnormals kept, overflow -> inf */
uint16_t oracle_f32_to_f16(float f) {
    uint32_t x = f2u(f);
    uint16_t sign = (uint16_t)((x >> 16) & 0x8000u);
    uint32_t ax = x & 0x7FFFFFFFu;
    if (ax > 0x7F800000u) return (uint16_t)(sign | 0x7E00u | ((ax >> 13) & 0x3FFu));
    if (ax >= 0x47800000u) return (uint16_t)(sign | 0x7C00u);          /* >= 65536 (and inf) */
    if (ax >= 0x38800000u) {                                             /* normal fp16 range */
        uint32_t e = (ax >> 23) - 127u + 15u;
        uint32_t m = ax & 0x7FFFFFu;
        uint32_t h = (e << 10) | (m >> 13);
        uint32_t rem = m & 0x1FFFu;
        if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;          /* may carry to inf */
        return (uint16_t)(sign | h);
    }
    /* subnormal / zero: units of 2^-24, exact scaling then RNE */
    float m = nearbyintf(u2f(ax) * 16777216.0f);
    return (uint16_t)(sign | (uint16_t)m);
}

float oracle_f16_to_f32(uint16_t h) {
    uint32_t sign = ((uint32_t)h & 0x8000u) << 16;
    uint32_t e = (h >> 10) & 0x1Fu, m = h & 0x3FFu;
    if (e == 0x1F) return u2f(sign | 0x7F800000u | (m << 13));
    if (e == 0) {
        float v = (float)m * (1.0f / 16777216.0f);
        return sign ? -v : v;
    }
    return u2f(sign | ((e - 15u + 127u) << 23) | (m << 13));
}

/* Round a compute-type value to the storage dtype and back. */
static inline double rn(double v, int dtype) {
    switch (dtype) {
    case AWQ_ORACLE_BF16: return (double)oracle_bf16_to_f32(oracle_f32_to_bf16((float)v));
    case AWQ_ORACLE_F16: return (double)oracle_f16_to_f32(oracle_f32_to_f16((float)v));
    case AWQ_ORACLE_F32: return (double)(float)v;
    default: return v;
    }
}

/* One binary op of the reference, evaluated the way torch CPU does for dtype D:
 * fp32 math for bf16/f16/f32 (the operands are exact fp32 values), fp64 for f64. */
static inline double op_add(double a, double b, int d) {
    if (d == AWQ_ORACLE_F64) return a + b;
    return rn((double)((float)a + (float)b), d);
}
static inline double op_sub(double a, double b, int d) {
    if (d == AWQ_ORACLE_F64) return a - b;
    return rn((double)((float)a - (float)b), d);
}
static inline double op_div(double a, double b, int d) {
    if (d == AWQ_ORACLE_F64) return a / b;
    return rn((double)((float)a / (float)b), d);
}
static inline double op_round(double a, int d) {            /* torch.round: half-to-even */
    if (d == AWQ_ORACLE_F64) return nearbyint(a);
    return rn((double)nearbyintf((float)a), d);
}
static inline double op_clamp(double a, double lo, double hi) {   /* NaN propagates */
    if (isnan(a)) return a;
    if (a < lo) a = lo;
    if (a > hi) a = hi;
    return a;
}
static inline int32_t to_i32(double v) {                    /* x86 cvtt: NaN -> INT_MIN */
    if (isnan(v)) return INT32_MIN;
    return (int32_t)v;
}

static inline double load_elem(const void* x, int dtype, int64_t i) {
    switch (dtype) {
    case AWQ_ORACLE_BF16: return (double)oracle_bf16_to_f32(((const uint16_t*)x)[i]);
    case AWQ_ORACLE_F16: return (double)oracle_f16_to_f32(((const uint16_t*)x)[i]);
    case AWQ_ORACLE_F32: return (double)((const float*)x)[i];
    default: return ((const double*)x)[i];
    }
}

/* fp16 bits of a NaN scale, as the reference's CPU ops leave them (awq.py:192-205, the fp32
 * scale buffer of awq.py:327/352, .to(float16) of awq.py:411).  Derived from the op chain and
 * pinned by every NaN scale of tests/golden/golden_nan.* (1 852 of them) and golden_small.*:
 *   - torch.min/max over n >= 2 elements holding a NaN return the all-ones NaN of the compute
 *     type (ATen's vectorised maximum/minimum OR the unordered-compare mask into the result);
 *     rounded to fp16 by the scalar c10 conversion that is 0xFE00, to bf16 0x7FC0; over n = 1
 *     they return the element itself;
 *   - abs clears the sign, Python max() keeps its first argument, fp32/fp64 a - b of two NaNs
 *     returns b (fp16, computed in fp32: a); inf - inf is the x86 default NaN (sign set);
 *   - bf16 rounding gives 0x7FC0 for any NaN; the fp16 -> fp32 store into the scale buffer
 *     (scales[c, g] = scale) gives 0x7FFFFFFF for any fp16 NaN; fp64 -> fp32 keeps the sign and
 *     the top mantissa bits; fp32 -> fp16 (awq.py:411) keeps the sign and the top 10 mantissa
 *     bits with the quiet bit set.
 * small = 1: the small-tensor path (awq.py:130-171), whose input-dtype scales go to fp16
 * directly (no fp32 buffer).  n = group length; has_nan = the group holds a NaN (else the NaN
 * came from inf - inf); e = bits of the group's NaN element (used when n == 1). */
uint16_t oracle_nan_scale_f16(int dtype, int sym, int small, int64_t n, int has_nan, uint64_t e) {
    switch (dtype) {
    case AWQ_ORACLE_BF16:
        return 0x7E00;
    case AWQ_ORACLE_F16:
        if (!small) return 0x7FFF;
        if (sym) return 0x7E00;
        return (n == 1 && has_nan) ? (uint16_t)((e & 0x8000u) | 0x7E00u) : 0xFE00;
    default: {
        if (!has_nan) return 0xFE00;
        if (n >= 2) return 0xFFFF;
        const int f64 = dtype == AWQ_ORACLE_F64;
        uint16_t sign = (uint16_t)(f64 ? (e >> 48) & 0x8000u : (e >> 16) & 0x8000u);
        uint16_t m10 = (uint16_t)(f64 ? (e >> 42) & 0x3FFu : (e >> 13) & 0x3FFu);
        if (sym) sign = 0x8000;
        return (uint16_t)(sign | 0x7E00u | m10);
    }
    }
}

static inline uint64_t load_bits(const void* x, int dtype, int64_t i) {
    switch (dtype) {
    case AWQ_ORACLE_BF16:
    case AWQ_ORACLE_F16: return ((const uint16_t*)x)[i];
    case AWQ_ORACLE_F32: return ((const uint32_t*)x)[i];
    default: return ((const uint64_t*)x)[i];
    }
}

static inline int bits_nan(uint64_t b, int dtype) {
    switch (dtype) {
    case AWQ_ORACLE_BF16: return (b & 0x7FFFu) > 0x7F80u;
    case AWQ_ORACLE_F16: return (b & 0x7FFFu) > 0x7C00u;
    case AWQ_ORACLE_F32: return (b & 0x7FFFFFFFu) > 0x7F800000u;
    default: return (b & 0x7FFFFFFFFFFFFFFFull) > 0x7FF0000000000000ull;
    }
}

/* fp16 bits of the scale of group [k0, k1) of row r (n = L elements incl. padding) */
static uint16_t scale_f16(double s, const void* x, int dtype, int64_t base, int64_t k0, int64_t k1, int64_t L,
                          int sym, int small) {
    if (!isnan(s)) return oracle_f32_to_f16((float)s);
    int has_nan = 0;
    uint64_t e = 0;
    for (int64_t k = k0; k < k1 && !has_nan; ++k) {
        uint64_t b = load_bits(x, dtype, base + k);
        if (bits_nan(b, dtype)) { has_nan = 1; e = b; }
    }
    return oracle_nan_scale_f16(dtype, sym, small, L, has_nan, e);
}

/* awq.py:173-213 — scale and zero point of one group (values already in compute type).
 * gpu = 1: as torch's GPU kernels evaluate these lines (device="cuda"): the division by the
 * Python int qmax - qmin is a product with the compute type's RN(1 / (qmax - qmin)) (ATen's
 * GPU division by a CPU scalar), and clamp(-0, 0, qmax) = +0 (IEEE maximum). */
static void group_scale_zp_dev(double mn, double mx, int dtype, int qmin, int qmax, int sym, int gpu,
                               double* s_out, double* z_out);
static void group_scale_zp(double mn, double mx, int dtype, int qmin, int qmax, int sym,
                           double* s_out, double* z_out) {
    group_scale_zp_dev(mn, mx, dtype, qmin, qmax, sym, 0, s_out, z_out);
}
static void group_scale_zp_dev(double mn, double mx, int dtype, int qmin, int qmax, int sym, int gpu,
                               double* s_out, double* z_out) {
    if (sym) {                                   /* awq.py:196-199, Python builtin max() */
        double amn = fabs(mn), amx = fabs(mx);
        double a = (amx > amn) ? amx : amn;
        mn = -a;
        mx = a;
    }
    double s;                                                                 /* awq.py:202 */
    if (!gpu) s = op_div(op_sub(mx, mn, dtype), (double)(qmax - qmin), dtype);
    else if (dtype == AWQ_ORACLE_F64) s = op_sub(mx, mn, dtype) * (1.0 / (double)(qmax - qmin));
    else s = rn((double)((float)op_sub(mx, mn, dtype) * (1.0f / (float)(qmax - qmin))), dtype);
    double lo = rn(1e-10, dtype);                                             /* awq.py:205 */
    if (!isnan(s) && s < lo) s = lo;
    double z;
    if (sym) {
        z = 0.0;                                                              /* awq.py:208 */
    } else {
        z = op_sub((double)qmin, op_div(mn, s, dtype), dtype);                /* awq.py:210 */
        z = op_clamp(op_round(z, dtype), qmin, qmax);                         /* awq.py:211 */
        if (gpu && z == 0.0) z = 0.0;                                         /* GPU clamp: +0 */
    }
    *s_out = s;
    *z_out = z;
}

int oracle_quantize(const void* x, int dtype, int64_t rows, int64_t K, int64_t L, int bits,
                    int sym, int32_t* tensor_q, uint16_t* scales_f16, int32_t* zeros) {
    return oracle_quantize_ex(x, dtype, rows, K, L, bits, sym, 0, tensor_q, scales_f16, zeros);
}

/* small = 1: the small-tensor path (awq.py:130-171, L = K): only NaN scale bits differ */
int oracle_quantize_ex(const void* x, int dtype, int64_t rows, int64_t K, int64_t L, int bits,
                       int sym, int small, int32_t* tensor_q, uint16_t* scales_f16, int32_t* zeros) {
    if (!x || rows < 0 || K < 0 || L <= 0 || (bits != 4 && bits != 8)) return -1;
    int qmin = sym ? -(1 << (bits - 1)) : 0;                                  /* awq.py:114-128 */
    int qmax = sym ? (1 << (bits - 1)) - 1 : (1 << bits) - 1;
    int64_t G = (K + L - 1) / L;
    /* rows are independent: OpenMP over rows (results do not depend on the thread count) */
#pragma omp parallel for schedule(static) if (rows * K >= (1 << 16))
    for (int64_t r = 0; r < rows; ++r) {
        for (int64_t g = 0; g < G; ++g) {
            int64_t k0 = g * L, k1 = k0 + L;
            int padded = k1 > K;                                              /* awq.py:337-339 */
            if (k1 > K) k1 = K;
            double mn = padded ? 0.0 : INFINITY, mx = padded ? 0.0 : -INFINITY;
            int nan = 0;
            for (int64_t k = k0; k < k1; ++k) {
                double v = load_elem(x, dtype, r * K + k);
                if (isnan(v)) nan = 1;
                if (v < mn) mn = v;
                if (v > mx) mx = v;
            }
            if (nan) { mn = NAN; mx = NAN; }
            double s, z;
            group_scale_zp(mn, mx, dtype, qmin, qmax, sym, &s, &z);
            if (scales_f16) scales_f16[r * G + g] = scale_f16(s, x, dtype, r * K, k0, k1, L, sym, small);
            if (zeros) zeros[r * G + g] = to_i32(z);
            if (tensor_q) {
                for (int64_t k = k0; k < k1; ++k) {
                    double v = load_elem(x, dtype, r * K + k);
                    double t = op_add(op_div(v, s, dtype), z, dtype);          /* awq.py:245 */
                    t = op_clamp(op_round(t, dtype), qmin, qmax);              /* awq.py:248 */
                    tensor_q[r * K + k] = to_i32(t);
                }
            }
        }
    }
    return 0;
}

/* awq.py:173-213 per group, the scale / zero point themselves (exact doubles of the dtype's
 * values): what _compute_scale_zp_for_group returns (0-d, dtype D) and, rounded to fp32,
 * what _quantize_per_group stores (awq.py:327-328, 352-353). */
int oracle_group_params_ex(const void* x, int dtype, int64_t rows, int64_t K, int64_t L, int bits, int sym, int gpu,
                           double* scales, double* zeros) {
    if (!x || rows < 0 || K < 0 || L <= 0 || (bits != 4 && bits != 8)) return -1;
    int qmin = sym ? -(1 << (bits - 1)) : 0;
    int qmax = sym ? (1 << (bits - 1)) - 1 : (1 << bits) - 1;
    int64_t G = (K + L - 1) / L;
    for (int64_t r = 0; r < rows; ++r) {
        for (int64_t g = 0; g < G; ++g) {
            int64_t k0 = g * L, k1 = k0 + L;
            int padded = k1 > K;
            if (k1 > K) k1 = K;
            double mn = padded ? 0.0 : INFINITY, mx = padded ? 0.0 : -INFINITY;
            int nan = 0;
            for (int64_t k = k0; k < k1; ++k) {
                double v = load_elem(x, dtype, r * K + k);
                if (isnan(v)) nan = 1;
                if (v < mn) mn = v;
                if (v > mx) mx = v;
            }
            if (nan) { mn = NAN; mx = NAN; }
            double s, z;
            group_scale_zp_dev(mn, mx, dtype, qmin, qmax, sym, gpu, &s, &z);
            if (scales) scales[r * G + g] = s;
            if (zeros) zeros[r * G + g] = z;
        }
    }
    return 0;
}

int oracle_group_params(const void* x, int dtype, int64_t rows, int64_t K, int64_t L, int bits, int sym,
                        double* scales, double* zeros) {
    return oracle_group_params_ex(x, dtype, rows, K, L, bits, sym, 0, scales, zeros);
}


/* awq.py:215-250 (_quantize_tensor, mode 0) and awq.py:252-284 (_dequantize_tensor, mode 1)
 * with given per-group parameters (double), which enter each op in its compute type (fp32;
 * fp64 for D = f64) unrounded to D, as torch's CPU kernels use a 0-d operand's original
 * value; out in dtype D (bf16 / f16 bits, f32, f64). */
static inline void store_elem(void* out, int dtype, int64_t i, double v) {
    switch (dtype) {
    case AWQ_ORACLE_BF16: ((uint16_t*)out)[i] = oracle_f32_to_bf16((float)v); break;
    case AWQ_ORACLE_F16: ((uint16_t*)out)[i] = oracle_f32_to_f16((float)v); break;
    case AWQ_ORACLE_F32: ((float*)out)[i] = (float)v; break;
    default: ((double*)out)[i] = v;
    }
}
int oracle_apply_params(const void* x, int dtype, int64_t rows, int64_t K, int64_t L, const double* scales,
                        const double* zeros, int qmin, int qmax, int mode, void* out) {
    if (!x || !scales || !zeros || !out || rows < 0 || K < 0 || L <= 0) return -1;
    int64_t G = (K + L - 1) / L;
    for (int64_t r = 0; r < rows; ++r) {
        for (int64_t k = 0; k < K; ++k) {
            int64_t gi = r * G + k / L;
            double s = scales[gi], z = zeros[gi];
            if (dtype != AWQ_ORACLE_F64) { s = (double)(float)s; z = (double)(float)z; }
            double v = load_elem(x, dtype, r * K + k), t;
            if (mode == 0) {
                t = op_add(op_div(v, s, dtype), z, dtype);                 /* awq.py:245 */
                t = op_clamp(op_round(t, dtype), qmin, qmax);              /* awq.py:248 */
            } else {
                t = op_sub(v, z, dtype);                                   /* awq.py:282 */
                t = (dtype == AWQ_ORACLE_F64) ? t * s : rn((double)((float)t * (float)s), dtype);
            }
            store_elem(out, dtype, r * K + k, t);
        }
    }
    return 0;
}

/* awq.py:245 and awq.py:282 under torch's type promotion (round 5; integer tensors round 6):
 * the two ops of
 *   mode 0  round(tensor / scale + zero_point).clamp(qmin, qmax)
 *   mode 1  (tensor_q - zero_point) * scale
 * are evaluated in their own result dtypes d1 (first op) and d2 (second op) — torch's
 * result_type of the operands — one element per parameter (the caller has broadcast
 * everything to the result's shape).  An operand of another dtype is converted to the op's
 * dtype first (c10::convert: an integer to bf16 / fp16 through fp32, i.e. RN_f32 of the
 * exact integer, then RN to the op dtype; to an integer dtype by truncation to its width),
 * EXCEPT a one-element parameter of a bf16 / fp16 op (flags bit 0: scale, bit 1:
 * zero_point), which ATen's reduced-float CPU kernels read at its original value in fp32
 * (TensorIterator::original_scalar_value) — checked against torch on CPU by
 * tests/golden/golden_promote*.* (reference calls).  Integer ops wrap at their width, like
 * torch's integer kernels.
 * Dtype codes: the four float codes, AWQ_ORACLE_I32 .. AWQ_ORACLE_U8 (tensor and op dtypes),
 * AWQ_ORACLE_BOOL / U16 / U32 / U64 (tensor dtypes only: torch has no such op here).
 * Parameters: doubles (exact float values), or — flags bit 2 (scale) / bit 3 (zero_point) —
 * int64 values in the same arrays (bit 4 / 5: those int64 words are uint64).  Bit 6: torch's
 * GPU clamp (IEEE maximum: clamp(-0, 0, qmax) = +0; the CPU clamp keeps the -0), with bits 0 / 1
 * clear — the reference evaluated with device="cuda". */
typedef struct { double f; int64_t i; int kind; } oval;     /* kind 0 float, 1 int64, 2 uint64 */
static inline int is_int_code(int d) { return d >= AWQ_ORACLE_I32; }
static inline oval of_f(double f) { oval v = {f, 0, 0}; return v; }
static inline oval of_i(int64_t i, int kind) { oval v = {0.0, i, kind}; return v; }
static oval load_val(const void* x, int dtype, int64_t i) {
    switch (dtype) {
    case AWQ_ORACLE_I32: return of_i(((const int32_t*)x)[i], 1);
    case AWQ_ORACLE_I64: return of_i(((const int64_t*)x)[i], 1);
    case AWQ_ORACLE_I16: return of_i(((const int16_t*)x)[i], 1);
    case AWQ_ORACLE_I8: return of_i(((const int8_t*)x)[i], 1);
    case AWQ_ORACLE_U8: return of_i(((const uint8_t*)x)[i], 1);
    case AWQ_ORACLE_BOOL: return of_i(((const uint8_t*)x)[i] != 0, 1);
    case AWQ_ORACLE_U16: return of_i(((const uint16_t*)x)[i], 1);
    case AWQ_ORACLE_U32: return of_i(((const uint32_t*)x)[i], 1);
    case AWQ_ORACLE_U64: return of_i(((const int64_t*)x)[i], 2);
    default: return of_f(load_elem(x, dtype, i));
    }
}
static inline int64_t wrap_to(uint64_t v, int d) {           /* truncation to d's width */
    switch (d) {
    case AWQ_ORACLE_I32: return (int32_t)(uint32_t)v;
    case AWQ_ORACLE_I16: return (int16_t)(uint16_t)v;
    case AWQ_ORACLE_I8: return (int8_t)(uint8_t)v;
    case AWQ_ORACLE_U8: return (uint8_t)v;
    default: return (int64_t)v;
    }
}
static inline float int_to_f32(oval v) { return v.kind == 2 ? (float)(uint64_t)v.i : (float)v.i; }
static oval convert_val(oval v, int d) {
    if (is_int_code(d)) {
        if (v.kind) return of_i(wrap_to((uint64_t)v.i, d), 1);
        return of_i(wrap_to((uint64_t)(int64_t)v.f, d), 1);       /* not reached by torch's promotion */
    }
    if (v.kind == 0) return of_f(d == AWQ_ORACLE_F64 ? v.f : rn((double)(float)v.f, d));
    if (d == AWQ_ORACLE_F64) return of_f(v.kind == 2 ? (double)(uint64_t)v.i : (double)v.i);
    return of_f(rn((double)int_to_f32(v), d));
}
static oval param_val(const double* a, int64_t i, int is_int, int is_unsigned) {
    if (!is_int) return of_f(a[i]);
    int64_t w;
    memcpy(&w, &a[i], 8);
    return of_i(w, is_unsigned ? 2 : 1);
}
static oval enter_val(oval v, int d, int one_element) {
    if (one_element && (d == AWQ_ORACLE_BF16 || d == AWQ_ORACLE_F16))
        return of_f(v.kind ? (double)int_to_f32(v) : (double)(float)v.f);
    return convert_val(v, d);
}
static oval op2v(char op, oval a, oval b, int d) {               /* a, b already in dtype d */
    if (is_int_code(d)) {
        uint64_t ua = (uint64_t)a.i, ub = (uint64_t)b.i;
        return of_i(wrap_to(op == '-' ? ua - ub : op == '*' ? ua * ub : ua + ub, d), 1);
    }
    if (d == AWQ_ORACLE_F64)
        return of_f(op == '/' ? a.f / b.f : op == '-' ? a.f - b.f : op == '*' ? a.f * b.f : a.f + b.f);
    float fa = (float)a.f, fb = (float)b.f;
    float r = op == '/' ? fa / fb : op == '-' ? fa - fb : op == '*' ? fa * fb : fa + fb;
    return of_f(rn((double)r, d));
}
static void store_val(void* out, int d, int64_t i, oval v) {
    switch (d) {
    case AWQ_ORACLE_I32: ((int32_t*)out)[i] = (int32_t)v.i; break;
    case AWQ_ORACLE_I64: ((int64_t*)out)[i] = v.i; break;
    case AWQ_ORACLE_I16: ((int16_t*)out)[i] = (int16_t)v.i; break;
    case AWQ_ORACLE_I8: ((int8_t*)out)[i] = (int8_t)v.i; break;
    case AWQ_ORACLE_U8: ((uint8_t*)out)[i] = (uint8_t)v.i; break;
    default: store_elem(out, d, i, v.f);
    }
}
int oracle_apply_params_ex(const void* x, int xdt, int64_t n, const double* scales, const double* zeros, int qmin,
                           int qmax, int mode, int d1, int d2, int flags, void* out) {
    if (!x || !scales || !zeros || !out || n < 0 || xdt < 0 || xdt > AWQ_ORACLE_U64 || d1 < 0 ||
        d1 > AWQ_ORACLE_U8 || d2 < 0 || d2 > AWQ_ORACLE_U8 || (mode == 0 && (is_int_code(d1) || is_int_code(d2))) ||
        (flags & ~127))
        return -1;
    for (int64_t i = 0; i < n; ++i) {
        oval v = convert_val(load_val(x, xdt, i), d1), t;
        oval s = param_val(scales, i, flags & 4, flags & 16), z = param_val(zeros, i, flags & 8, flags & 32);
        if (mode == 0) {
            t = op2v('/', v, enter_val(s, d1, flags & 1), d1);                          /* awq.py:245 */
            t = op2v('+', convert_val(t, d2), enter_val(z, d2, flags & 2), d2);
            t.f = op_clamp(op_round(t.f, d2), qmin, qmax);                              /* awq.py:248 */
            if ((flags & 64) && t.f == 0.0 && qmin == 0) t.f = 0.0;   /* GPU clamp: max(-0, +0) = +0 */
        } else {
            t = op2v('-', v, enter_val(z, d1, flags & 2), d1);                          /* awq.py:282 */
            t = op2v('*', convert_val(t, d2), enter_val(s, d2, flags & 1), d2);
        }
        store_val(out, d2, i, t);
    }
    return 0;
}

/* Opt-in clip search (scale_method="search").  NOT in the reference (it stores
 * scale_method, awq.py:66, validates it, :111-112, and never reads it again), so this
 * restates the product's own definition (include/awq_hip.h, awq_quantize_search) — parity
 * between it and the HIP kernel is checked, parity with the reference is unpinned except
 * for candidate 0, which IS the RTN path above (golden-pinned).
 *
 * Per group: mn/mx as in oracle_quantize; sym -> (-a, a) with a = Python max(|mn|,|mx|);
 * candidate i scales both ends by alpha_i = (n_grid - i) / n_grid (computed in the compute
 * type, product rounded to D), takes (s, z) by awq.py:202-211, quantizes every element
 * (awq.py:245-248) and dequantizes it the reference's way (awq.py:459-539:
 * fp16(fp16(q - z) * fp16(s))).  err = sum (x - dq)^2 in the compute type, summed in the
 * product's canonical order: chunk l (0..63) = elements k0+8l .. k0+8l+7 accumulated in
 * sequence, then the pairwise tree over the 64 chunks, adjacent pairs first (written as an
 * xor butterfly t[l] = a[l] + a[l^o], o = 1, 2, .., 32, which every lane of the GPU's wave
 * reproduces).
 * Smallest err wins, ties -> smaller i; NaN groups skip the search.  L <= 512. */
static double cadd(double a, double b, int f64) { return f64 ? a + b : (double)((float)a + (float)b); }
static double cmul(double a, double b, int f64) { return f64 ? a * b : (double)((float)a * (float)b); }
static double csub(double a, double b, int f64) { return f64 ? a - b : (double)((float)a - (float)b); }

static double tree_sum64(double* a, int f64) {
    double t[64];
    for (int o = 1; o < 64; o <<= 1) {   /* pairwise tree over adjacent chunks */
        for (int l = 0; l < 64; ++l) t[l] = cadd(a[l], a[l ^ o], f64);
        memcpy(a, t, sizeof t);
    }
    return a[0];
}

int oracle_quantize_search(const void* x, int dtype, int64_t rows, int64_t K, int64_t L, int bits,
                           int sym, int n_grid, int n_cand, int32_t* tensor_q, uint16_t* scales_f16,
                           int32_t* zeros) {
    return oracle_quantize_search_ex(x, dtype, rows, K, L, bits, sym, 0, n_grid, n_cand, tensor_q, scales_f16,
                                     zeros);
}

int oracle_quantize_search_ex(const void* x, int dtype, int64_t rows, int64_t K, int64_t L, int bits,
                              int sym, int small, int n_grid, int n_cand, int32_t* tensor_q, uint16_t* scales_f16,
                              int32_t* zeros) {
    if (!x || rows < 0 || K < 0 || L <= 0 || (bits != 4 && bits != 8)) return -1;
    if (n_grid < 1 || n_cand < 1 || n_cand > n_grid) return -1;
    if (L > 512 && K > 512) return -1;   /* one 8-element chunk per slot, 64 slots */
    int qmin = sym ? -(1 << (bits - 1)) : 0;
    int qmax = sym ? (1 << (bits - 1)) - 1 : (1 << bits) - 1;
    int f64 = dtype == AWQ_ORACLE_F64;
    int64_t G = (K + L - 1) / L;
#pragma omp parallel for schedule(static) if (rows * K >= (1 << 14))
    for (int64_t r = 0; r < rows; ++r) {
        for (int64_t g = 0; g < G; ++g) {
            int64_t k0 = g * L, k1 = k0 + L;
            int padded = k1 > K;
            if (k1 > K) k1 = K;
            double mn = padded ? 0.0 : INFINITY, mx = padded ? 0.0 : -INFINITY;
            int nan = 0;
            for (int64_t k = k0; k < k1; ++k) {
                double v = load_elem(x, dtype, r * K + k);
                if (isnan(v)) nan = 1;
                if (v < mn) mn = v;
                if (v > mx) mx = v;
            }
            if (nan) { mn = NAN; mx = NAN; }
            if (!nan) {
                if (sym) {
                    double a = (fabs(mx) > fabs(mn)) ? fabs(mx) : fabs(mn);
                    mn = -a;
                    mx = a;
                }
                double best = INFINITY;
                int bi = 0;
                for (int i = 0; i < n_cand; ++i) {
                    double al = f64 ? (double)(n_grid - i) / (double)n_grid
                                    : (double)((float)(n_grid - i) / (float)n_grid);
                    double cs, cz;
                    group_scale_zp(rn(cmul(mn, al, f64), dtype), rn(cmul(mx, al, f64), dtype), dtype, qmin,
                                   qmax, sym, &cs, &cz);
                    float sh = oracle_f16_to_f32(oracle_f32_to_f16((float)cs));
                    double acc[64];
                    for (int l = 0; l < 64; ++l) {
                        acc[l] = 0.0;
                        int64_t c0 = k0 + 8 * l, c1 = c0 + 8 < k1 ? c0 + 8 : k1;
                        for (int64_t k = c0; k < c1; ++k) {
                            double v = load_elem(x, dtype, r * K + k);
                            double q = op_add(op_div(v, cs, dtype), cz, dtype);
                            q = op_clamp(op_round(q, dtype), qmin, qmax);
                            float h = oracle_f16_to_f32(oracle_f32_to_f16((float)(q - cz)));
                            double dq = (double)oracle_f16_to_f32(oracle_f32_to_f16(h * sh));
                            double d = csub(v, dq, f64);
                            acc[l] = cadd(acc[l], cmul(d, d, f64), f64);
                        }
                    }
                    double err = tree_sum64(acc, f64);
                    if (err < best) { best = err; bi = i; }
                }
                double al = f64 ? (double)(n_grid - bi) / (double)n_grid
                                : (double)((float)(n_grid - bi) / (float)n_grid);
                mn = rn(cmul(mn, al, f64), dtype);
                mx = rn(cmul(mx, al, f64), dtype);
            }
            double s, z;
            group_scale_zp(mn, mx, dtype, qmin, qmax, sym, &s, &z);
            if (scales_f16) scales_f16[r * G + g] = scale_f16(s, x, dtype, r * K, k0, k1, L, sym, small);
            if (zeros) zeros[r * G + g] = to_i32(z);
            if (tensor_q) {
                for (int64_t k = k0; k < k1; ++k) {
                    double v = load_elem(x, dtype, r * K + k);
                    double t = op_add(op_div(v, s, dtype), z, dtype);
                    t = op_clamp(op_round(t, dtype), qmin, qmax);
                    tensor_q[r * K + k] = to_i32(t);
                }
            }
        }
    }
    return 0;
}

/* threads used by the OpenMP row loops (bench.py's cpu_baseline reports this count) */
int oracle_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
    return omp_get_max_threads();
#else
    (void)n;
    return 1;
#endif
}

/* awq.py:459-539: dq = (q - z) [int32] * scale [fp16 0-d]  -> fp16 math -> stored fp32.
 * NaN bits: the fp16 product keeps the scale's NaN (inf * 0: the default NaN 0xFE00); the
 * group's n = min(L, K - g L) results are copied into the fp32 output by ATen's fp16 -> fp32
 * copy (awq.py:527/531), which widens 8-element vectors bit-preservingly and converts the last
 * n % 8 elements one by one, turning any NaN into 0x7FFFFFFF (pinned: golden_nan.* .dq). */
int oracle_dequantize(const int32_t* tensor_q, const uint16_t* scales_f16, const int32_t* zeros,
                      int64_t rows, int64_t K, int64_t L, float* out) {
    if (!tensor_q || !scales_f16 || !zeros || !out || L <= 0) return -1;
    int64_t G = (K + L - 1) / L;
    for (int64_t r = 0; r < rows; ++r) {
        for (int64_t k = 0; k < K; ++k) {
            int64_t g = k / L;
            int32_t diff = (int32_t)((uint32_t)tensor_q[r * K + k] - (uint32_t)zeros[r * G + g]);
            float h = oracle_f16_to_f32(oracle_f32_to_f16((float)diff));
            float s = oracle_f16_to_f32(scales_f16[r * G + g]);
            float v = oracle_f16_to_f32(oracle_f32_to_f16(h * s));
            int64_t n = K - g * L < L ? K - g * L : L;
            if (isnan(v) && k - g * L >= (n & ~(int64_t)7)) v = u2f(0x7FFFFFFFu);
            out[r * K + k] = v;
        }
    }
    return 0;
}

/* Row-major pack used by the product's packed outputs (no reference counterpart:
 * the reference returns unpacked int32).  nibble/byte j of word c holds
 * (v[c*per + j] - qmin) masked to `bits`; positions past n are 0. */
int oracle_pack_rows(const int32_t* v, int64_t rows, int64_t n, int bits, int qmin, int32_t* packed) {
    if (!v || !packed || (bits != 4 && bits != 8)) return -1;
    int per = 32 / bits;
    uint32_t mask = (1u << bits) - 1u;
    int64_t words = (n + per - 1) / per;
    for (int64_t r = 0; r < rows; ++r) {
        for (int64_t c = 0; c < words; ++c) {
            uint32_t w = 0;
            for (int j = 0; j < per; ++j) {
                int64_t i = c * per + j;
                if (i < n) w |= (((uint32_t)v[r * n + i] - (uint32_t)qmin) & mask) << (bits * j);
            }
            packed[r * words + c] = (int32_t)w;
        }
    }
    return 0;
}

/* ---------------- activation-aware scale search (scale_method="awq") ----------------
 * NOT in the reference (awq.py:66 stores scale_method; no activations are collected):
 * restates the product's definition (include/awq_hip.h, awq_act_*), itself AutoAWQ's
 * published per-input-channel search (third-party; not vendored in the reference, not
 * installed here) with the output-MSE loss in its diagonal per-element form.  Parity with
 * the HIP kernels is checked bit for bit given the same scale table (the table's fp64
 * pow differs between math libraries by <= 1 fp32 ulp, checked separately); parity with
 * AutoAWQ is unpinned. */
#define ACT_ROW_BLOCK 256
#define ACT_ROW_SUB 32       /* rows per sub-block: a block sums its sub-blocks' sums */
#define ACT_GROUP_BLOCK 1024
#define ACT_GROUP_SUB 64     /* groups per sub-block of a loss block */
#define ACT_SUPER_BLOCKS 32  /* loss blocks per super-block of a candidate's total */

static inline float load_f(const void* x, int dtype, int64_t i) { return (float)load_elem(x, dtype, i); }

int oracle_act_stats(const void* x, int dtype, int64_t T, int64_t K, float* x_mean, float* x_sq) {
    if (!x || T <= 0 || K <= 0 || dtype == AWQ_ORACLE_F64) return -1;
    int64_t nblk = (T + ACT_ROW_BLOCK - 1) / ACT_ROW_BLOCK;
#pragma omp parallel for schedule(static) if (T * K >= (1 << 16))
    for (int64_t k = 0; k < K; ++k) {
        double a = 0.0, q = 0.0;
        for (int64_t b = 0; b < nblk; ++b) {   /* fp64: tokens ascending inside a 32-token
                                                  sub-block, sub-blocks ascending inside a
                                                  256-token block, blocks ascending */
            double pa = 0.0, pq = 0.0;
            int64_t t1 = (b + 1) * ACT_ROW_BLOCK < T ? (b + 1) * ACT_ROW_BLOCK : T;
            for (int64_t u = b * ACT_ROW_BLOCK; u < t1; u += ACT_ROW_SUB) {   /* 32-token sub-blocks */
                double sa = 0.0, sq = 0.0;
                int64_t u1 = u + ACT_ROW_SUB < t1 ? u + ACT_ROW_SUB : t1;
                for (int64_t t = u; t < u1; ++t) {
                    double v = (double)load_f(x, dtype, t * K + k);
                    sa += fabs(v);
                    sq += v * v;
                }
                pa += sa;
                pq += sq;
            }
            a += pa;
            q += pq;
        }
        x_mean[k] = (float)(a / (double)T);
        x_sq[k] = (float)(q / (double)T);
    }
    return 0;
}

/* partial[b][k] for this linear's ceil(R/256) row blocks: sum fp32(|w| / fp32(gmax + 1e-6f)) */
int oracle_weight_colsum(const void* w, int dtype, int64_t R, int64_t K, int64_t L, double* partial) {
    if (!w || R <= 0 || K <= 0 || L <= 0 || K % L || dtype == AWQ_ORACLE_F64) return -1;
    int64_t G = K / L, nblk = (R + ACT_ROW_BLOCK - 1) / ACT_ROW_BLOCK;
    float* gmax = (float*)malloc(sizeof(float) * (size_t)(R * G));
    if (!gmax) return -1;
    for (int64_t r = 0; r < R; ++r)
        for (int64_t g = 0; g < G; ++g) {
            float m = 0.0f;
            int nan = 0;
            for (int64_t k = g * L; k < (g + 1) * L; ++k) {
                float a = fabsf(load_f(w, dtype, r * K + k));
                if (isnan(a)) nan = 1;
                if (a > m) m = a;
            }
            gmax[r * G + g] = nan ? NAN : m;
        }
    for (int64_t b = 0; b < nblk; ++b)
        for (int64_t k = 0; k < K; ++k) {
            double s = 0.0;
            int64_t r1 = (b + 1) * ACT_ROW_BLOCK < R ? (b + 1) * ACT_ROW_BLOCK : R;
            for (int64_t u = b * ACT_ROW_BLOCK; u < r1; u += ACT_ROW_SUB) {   /* as oracle_act_stats */
                double su = 0.0;
                int64_t u1 = u + ACT_ROW_SUB < r1 ? u + ACT_ROW_SUB : r1;
                for (int64_t r = u; r < u1; ++r) {
                    float den = gmax[r * G + k / L] + 1e-6f;
                    su += (double)(fabsf(load_f(w, dtype, r * K + k)) / den);
                }
                s += su;
            }
            partial[b * K + k] = s;
        }
    free(gmax);
    return 0;
}

int oracle_column_mean(const double* partial, int64_t nblk, int64_t K, double divisor, float* out) {
    if (!partial || !out || nblk <= 0 || K <= 0) return -1;
    for (int64_t k = 0; k < K; ++k) {
        double s = 0.0;
        for (int64_t b = 0; b < nblk; ++b) s += partial[b * K + k];
        out[k] = (float)(s / divisor);
    }
    return 0;
}

/* The scale table's power function as include/awq_hip.h defines it (round 5): not libm pow,
 * whose last bit differs between math libraries, but a fixed sequence of IEEE fp64 +, *, /,
 * fma and rint (this file is built with -ffp-contract=off, so the only fused ops are the
 * explicit fma() calls):
 *   ln x:  x = m 2^e, m in [sqrt(2)/2, sqrt(2)) (subnormal x rescaled by 2^54 first);
 *          f = (m - 1) / (m + 1); P = 1/25, then P = fma(P, f^2, 1/(2j+1)) for j = 11 .. 1;
 *          ln m = fma(2f * f^2, P, 2f); ln x = fma(e, LN2_HI, fma(e, LN2_LO, ln m))
 *   e^y:   k = rint(y * INV_LN2); t = fma(-k, LN2_LO, fma(-k, LN2_HI, y));
 *          p = 1, then p = fma(p, t / j, 1) for j = 15 .. 1; p * 2^k (k > 1023: p 2^1023 2^(k-1023);
 *          k < -1022: (p 2^(k+600)) 2^-600); y > 709.8 -> inf, y < -746 -> 0, NaN -> NaN
 *   x^r:   r == 0 -> 1; NaN or negative x -> NaN; 0 -> 0; inf -> inf; else e^(r * ln x) */
static const double DET_LN2_HI = 6.93147180369123816490e-01, DET_LN2_LO = 1.90821492927058770002e-10,
                    DET_INV_LN2 = 1.44269504088896338700e+00;

static double det_pow2(int n) {
    uint64_t b = (uint64_t)(n + 1023) << 52;
    double d;
    memcpy(&d, &b, 8);
    return d;
}

static double det_log(double x) {
    int e = 0;
    if (x < 0x1p-1022) { x *= 0x1p54; e = -54; }
    uint64_t u;
    memcpy(&u, &x, 8);
    e += (int)((u >> 52) & 0x7FF) - 1023;
    uint64_t mb = (u & 0xFFFFFFFFFFFFFull) | 0x3FF0000000000000ull;
    double m;
    memcpy(&m, &mb, 8);
    if (m > 1.4142135623730951) { m *= 0.5; e += 1; }
    double f = (m - 1.0) / (m + 1.0), f2 = f * f, P = 1.0 / 25.0;
    for (int j = 11; j >= 1; --j) P = fma(P, f2, 1.0 / (double)(2 * j + 1));
    double t = 2.0 * f;
    double lm = fma(t * f2, P, t);
    return fma((double)e, DET_LN2_HI, fma((double)e, DET_LN2_LO, lm));
}

static double det_exp(double y) {
    if (isnan(y)) return y;
    if (y > 709.8) return INFINITY;
    if (y < -746.0) return 0.0;
    double k = rint(y * DET_INV_LN2);
    double t = fma(-k, DET_LN2_LO, fma(-k, DET_LN2_HI, y));
    double p = 1.0;
    for (int j = 15; j >= 1; --j) p = fma(p, t / (double)j, 1.0);
    int ki = (int)k;
    if (ki > 1023) return (p * det_pow2(1023)) * det_pow2(ki - 1023);
    if (ki < -1022) return (p * det_pow2(ki + 600)) * det_pow2(-600);
    return p * det_pow2(ki);
}

static double det_pow(double x, double r) {
    if (r == 0.0) return 1.0;
    if (isnan(x) || x < 0.0) return NAN;
    if (x == 0.0) return 0.0;
    if (isinf(x)) return x;
    return det_exp(r * det_log(x));
}

static double act_raw(const float* x_mean, const float* w_mean, int64_t k, double r) {
    double s = det_pow((double)x_mean[k], r);
    if (w_mean) s = s / (det_pow((double)w_mean[k], 1.0 - r) + 1e-4);
    return s < 1e-4 ? 1e-4 : s;   /* NaN stays NaN */
}

/* exported for the tests: det_pow against libm pow */
double oracle_det_pow(double x, double r) { return det_pow(x, r); }

int oracle_act_scale_table(const float* x_mean, const float* w_mean, int64_t K, int n_grid, float* table) {
    if (!x_mean || !table || K <= 0 || n_grid < 1) return -1;
    for (int i = 0; i < n_grid; ++i) {
        double r = (double)i / (double)n_grid, mx = -INFINITY, mn = INFINITY;
        int nan = 0;
        for (int64_t k = 0; k < K; ++k) {
            double s = act_raw(x_mean, w_mean, k, r);
            if (isnan(s)) nan = 1;
            if (s > mx) mx = s;
            if (s < mn) mn = s;
        }
        double norm = nan ? NAN : sqrt(mx * mn);
        for (int64_t k = 0; k < K; ++k) {
            double s = act_raw(x_mean, w_mean, k, r) / norm;
            if (isnan(s) || isinf(s)) s = 1.0;
            table[(int64_t)i * K + k] = (float)s;
        }
    }
    return 0;
}

int oracle_act_search_losses(const void* w, int dtype, int64_t R, int64_t K, int64_t L, int bits, int sym,
                             const float* table, int n_grid, const float* x_sq, float* part, int64_t stride) {
    if (!w || !table || !x_sq || !part || R <= 0 || K <= 0 || L < 8 || L > 512 || (L & (L - 1)) || K % L ||
        (bits != 4 && bits != 8) || dtype == AWQ_ORACLE_F64)
        return -1;
    int qmin = sym ? -(1 << (bits - 1)) : 0;
    int qmax = sym ? (1 << (bits - 1)) - 1 : (1 << bits) - 1;
    int64_t G = K / L;
    int lpg = (int)(L / 8);
#pragma omp parallel for schedule(static) if (R * K >= (1 << 12))
    for (int64_t r = 0; r < R; ++r) {
        float v[512], ws[512];
        for (int64_t g = 0; g < G; ++g) {
            int64_t k0 = g * L;
            for (int64_t e = 0; e < L; ++e) v[e] = load_f(w, dtype, r * K + k0 + e);
            for (int i = 0; i < n_grid; ++i) {
                const float* s = table + (int64_t)i * K + k0;
                double mn = INFINITY, mx = -INFINITY;
                int nan = 0;
                for (int64_t e = 0; e < L; ++e) {
                    ws[e] = (float)rn((double)(v[e] * s[e]), dtype);
                    if (isnan(ws[e])) nan = 1;
                    if (ws[e] < mn) mn = ws[e];
                    if (ws[e] > mx) mx = ws[e];
                }
                if (nan) { mn = NAN; mx = NAN; }
                double cs, cz;
                group_scale_zp(mn, mx, dtype, qmin, qmax, sym, &cs, &cz);
                float sh = oracle_f16_to_f32(oracle_f32_to_f16((float)cs));
                double acc[64];
                for (int l = 0; l < lpg; ++l) {   /* chunk l: elements 8l .. 8l+7 in order */
                    float a = 0.0f;
                    for (int j = 0; j < 8; ++j) {
                        int64_t e = 8 * l + j;
                        double q = op_add(op_div(ws[e], cs, dtype), cz, dtype);
                        q = op_clamp(op_round(q, dtype), qmin, qmax);
                        float hq = oracle_f16_to_f32(oracle_f32_to_f16((float)(q - cz)));
                        float dq = oracle_f16_to_f32(oracle_f32_to_f16(hq * sh));
                        float d = dq / s[e] - v[e];
                        a = a + x_sq[k0 + e] * (d * d);
                    }
                    acc[l] = a;
                }
                for (int o = 1; o < lpg; o <<= 1) {   /* pairwise tree, adjacent chunks first */
                    double t[64];
                    for (int l = 0; l < lpg; ++l) t[l] = (double)((float)acc[l] + (float)acc[l ^ o]);
                    memcpy(acc, t, sizeof(double) * (size_t)lpg);
                }
                part[(int64_t)i * stride + r * G + g] = (float)acc[0];
            }
        }
    }
    return 0;
}

int oracle_act_search_select(const float* part, int n_grid, int64_t stride, double* losses, int32_t* best) {
    if (!part || n_grid < 1 || stride <= 0) return -1;
    int64_t nblk = (stride + ACT_GROUP_BLOCK - 1) / ACT_GROUP_BLOCK;
    double bv = INFINITY;
    int bi = 0;
    for (int i = 0; i < n_grid; ++i) {
        /* fp64, three levels: groups ascending inside a 64-group sub-block; sub-blocks
         * ascending inside a 1024-group block; blocks ascending inside a 32-block super-block;
         * super-blocks ascending */
        double tot = 0.0;
        for (int64_t sb = 0; sb < nblk; sb += ACT_SUPER_BLOCKS) {
            double ss = 0.0;
            int64_t b1 = sb + ACT_SUPER_BLOCKS < nblk ? sb + ACT_SUPER_BLOCKS : nblk;
            for (int64_t b = sb; b < b1; ++b) {
                double s = 0.0;
                int64_t g1 = (b + 1) * ACT_GROUP_BLOCK < stride ? (b + 1) * ACT_GROUP_BLOCK : stride;
                for (int64_t u = b * ACT_GROUP_BLOCK; u < g1; u += ACT_GROUP_SUB) {
                    double su = 0.0;
                    int64_t u1 = u + ACT_GROUP_SUB < g1 ? u + ACT_GROUP_SUB : g1;
                    for (int64_t g = u; g < u1; ++g) su += (double)part[(int64_t)i * stride + g];
                    s += su;
                }
                ss += s;
            }
            tot += ss;
        }
        if (losses) losses[i] = tot;
        if (tot < bv) { bv = tot; bi = i; }
    }
    if (best) *best = bi;
    return 0;
}

/* out = RN_D(w * s[k]) in the weight dtype (bits of bf16 / fp16, or fp32) */
int oracle_apply_input_scale(const void* w, int dtype, int64_t R, int64_t K, const float* s, void* out) {
    if (!w || !s || !out || dtype == AWQ_ORACLE_F64) return -1;
    for (int64_t i = 0; i < R * K; ++i) {
        float y = load_f(w, dtype, i) * s[i % K];
        if (dtype == AWQ_ORACLE_BF16) ((uint16_t*)out)[i] = oracle_f32_to_bf16(y);
        else if (dtype == AWQ_ORACLE_F16) ((uint16_t*)out)[i] = oracle_f32_to_f16(y);
        else ((float*)out)[i] = y;
    }
    return 0;
}
