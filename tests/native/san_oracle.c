/* ASan/UBSan run of the CPU oracle (oracle/awq_oracle.c) — SURVEY.md §5 "sanitizers on the
 * CPU restatement".  TEST INFRASTRUCTURE: exercises every oracle entry point on edge shapes
 * (one element, one group, ragged tails, K % 8 != 0, one-element groups, groups longer than
 * the row, large group counts) and special values (NaN payloads, +-inf, subnormals, signed
 * zeros, huge magnitudes) for every dtype, bits 4 / 8, sym / asym, small-tensor flag on /
 * off.  Any out-of-bounds access, leak or undefined behaviour aborts the run (non-zero exit);
 * the results themselves are checked elsewhere (tests/test_oracle_golden.py). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/awq_oracle.h"

static uint64_t rng = 88172645463325252ull;
static uint64_t next(void) { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return rng; }

static void* make_input(int dtype, int64_t n) {
    const size_t es = dtype == AWQ_ORACLE_F64 ? 8 : dtype == AWQ_ORACLE_F32 ? 4 : 2;
    unsigned char* p = (unsigned char*)malloc(es * (size_t)(n > 0 ? n : 1));
    for (int64_t i = 0; i < n; ++i) {
        double v = ((double)(next() % 20001) - 10000.0) / 3000.0;
        switch (next() % 23) {
        case 0: v = NAN; break;
        case 1: v = INFINITY; break;
        case 2: v = -INFINITY; break;
        case 3: v = -0.0; break;
        case 4: v = 3e38; break;
        case 5: v = 1e-40; break;
        default: break;
        }
        if (dtype == AWQ_ORACLE_F64) ((double*)p)[i] = v;
        else if (dtype == AWQ_ORACLE_F32) ((float*)p)[i] = (float)v;
        else if (dtype == AWQ_ORACLE_F16) ((uint16_t*)p)[i] = oracle_f32_to_f16((float)v);
        else ((uint16_t*)p)[i] = oracle_f32_to_bf16((float)v);
        if (next() % 97 == 0 && dtype != AWQ_ORACLE_F64 && dtype != AWQ_ORACLE_F32)   /* NaN payloads */
            ((uint16_t*)p)[i] = (uint16_t)(0x7C01u | (next() & 0x83FFu)) | (dtype == AWQ_ORACLE_BF16 ? 0x7F80u : 0);
    }
    return p;
}

int main(void) {
    static const int64_t shapes[][3] = {   /* rows, K, L */
        {1, 1, 1}, {1, 1, 128}, {3, 1, 1}, {2, 7, 3}, {4, 128, 128}, {5, 300, 128}, {3, 203, 100}, {2, 1000, 64},
        {1, 4096, 4096}, {6, 12, 1}, {2, 130, 2}, {3, 513, 512}, {1, 9, 600}, {0, 16, 8}, {4, 0, 8}};
    long calls = 0;
    for (int dt = 0; dt < 4; ++dt)
        for (size_t si = 0; si < sizeof shapes / sizeof shapes[0]; ++si) {
            const int64_t R = shapes[si][0], K = shapes[si][1], L = shapes[si][2];
            const int64_t G = K > 0 ? (K + L - 1) / L : 0;
            void* x = make_input(dt, R * K);
            int32_t* tq = (int32_t*)malloc(sizeof(int32_t) * (size_t)(R * K + 1));
            uint16_t* sc = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)(R * G + 1));
            int32_t* zp = (int32_t*)malloc(sizeof(int32_t) * (size_t)(R * G + 1));
            double* s64 = (double*)malloc(sizeof(double) * (size_t)(R * G + 1));
            double* z64 = (double*)malloc(sizeof(double) * (size_t)(R * G + 1));
            float* dq = (float*)malloc(sizeof(float) * (size_t)(R * K + 1));
            void* out = make_input(dt, R * K);
            for (int bits = 4; bits <= 8; bits += 4)
                for (int sym = 0; sym < 2; ++sym)
                    for (int small = 0; small < 2; ++small) {
                        if (R * K == 0) continue;
                        oracle_quantize_ex(x, dt, R, K, L, bits, sym, small, tq, sc, zp);
                        if (L <= 512 || K <= 512)
                            oracle_quantize_search_ex(x, dt, R, K, L, bits, sym, small, 10, 5, tq, sc, zp);
                        oracle_dequantize(tq, sc, zp, R, K, L, dq);
                        oracle_group_params(x, dt, R, K, L, bits, sym, s64, z64);
                        const int qmin = sym ? -(1 << (bits - 1)) : 0, qmax = sym ? (1 << (bits - 1)) - 1 : (1 << bits) - 1;
                        oracle_apply_params(x, dt, R, K, L, s64, z64, qmin, qmax, 0, out);
                        oracle_apply_params(x, dt, R, K, L, s64, z64, qmin, qmax, 1, out);
                        int32_t* packed = (int32_t*)malloc(sizeof(int32_t) * (size_t)(R * ((K * bits + 31) / 32) + 1));
                        oracle_pack_rows(tq, R, K, bits, qmin, packed);
                        free(packed);
                        for (int has = 0; has < 2; ++has)
                            oracle_nan_scale_f16(dt, sym, small, L, has, next());
                        calls += 9;
                    }
            free(x); free(tq); free(sc); free(zp); free(s64); free(z64); free(dq); free(out);
        }
    /* activation-aware search: T tokens x K, linears of R rows, groups of L (power of two) */
    for (int dt = 0; dt < 3; ++dt) {
        const int64_t T = 37, K = 256, R = 40, L = 64;
        void* xa = make_input(dt, T * K);
        void* w = make_input(dt, R * K);
        float *xm = malloc(sizeof(float) * K), *xs = malloc(sizeof(float) * K), *wm = malloc(sizeof(float) * K);
        oracle_act_stats(xa, dt, T, K, xm, xs);
        for (int64_t k = 0; k < K; ++k) { if (!(xm[k] == xm[k])) xm[k] = 1.f; if (!(xs[k] == xs[k])) xs[k] = 1.f; }
        double* part = malloc(sizeof(double) * (size_t)(((R + 255) / 256) * K));
        oracle_weight_colsum(w, dt, R, K, L, part);
        oracle_column_mean(part, (R + 255) / 256, K, (double)R, wm);
        const int ng = 8;
        float* table = malloc(sizeof(float) * ng * K);
        oracle_act_scale_table(xm, wm, K, ng, table);
        oracle_act_scale_table(xm, NULL, K, ng, table);
        const int64_t stride = R * (K / L);
        float* losses_part = malloc(sizeof(float) * ng * stride);
        oracle_act_search_losses(w, dt, R, K, L, 4, 0, table, ng, xs, losses_part, stride);
        double* losses = malloc(sizeof(double) * ng);
        int32_t best = -1;
        oracle_act_search_select(losses_part, ng, stride, losses, &best);
        void* scaled = make_input(dt, R * K);
        oracle_apply_input_scale(w, dt, R, K, table, scaled);
        free(xa); free(w); free(xm); free(xs); free(wm); free(part); free(table); free(losses_part); free(losses);
        free(scaled);
        calls += 8;
    }
    printf("san_oracle: %ld calls clean\n", calls);
    return 0;
}
