/* awq_oracle.h — CPU restatement of the reference quantizer (TEST INFRASTRUCTURE ONLY).
 * See awq_oracle.c for the reference file:line each function follows. */
#ifndef AWQ_ORACLE_H
#define AWQ_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
enum { AWQ_ORACLE_BF16 = 0, AWQ_ORACLE_F16 = 1, AWQ_ORACLE_F32 = 2, AWQ_ORACLE_F64 = 3 };

/* x: [rows, K] row-major in `dtype`; groups of L along K, tail zero-padded (L >= K: one group).
 * Outputs (any may be NULL): tensor_q int32 [rows, K], scales fp16 bits [rows, G], zeros int32 [rows, G]. */
int oracle_quantize(const void* x, int dtype, int64_t rows, int64_t K, int64_t L, int bits, int sym,
                    int32_t* tensor_q, uint16_t* scales_f16, int32_t* zeros);
/* small = 1: the small-tensor path (awq.py:130-171); only the bits of NaN scales differ */
int oracle_quantize_ex(const void* x, int dtype, int64_t rows, int64_t K, int64_t L, int bits, int sym, int small,
                       int32_t* tensor_q, uint16_t* scales_f16, int32_t* zeros);
uint16_t oracle_nan_scale_f16(int dtype, int sym, int small, int64_t n, int has_nan, uint64_t e);
int oracle_quantize_search_ex(const void* x, int dtype, int64_t rows, int64_t K, int64_t L, int bits, int sym,
                              int small, int n_grid, int n_cand, int32_t* tensor_q, uint16_t* scales_f16,
                              int32_t* zeros);
/* opt-in clip search (product definition, include/awq_hip.h awq_quantize_search) */
int oracle_quantize_search(const void* x, int dtype, int64_t rows, int64_t K, int64_t L, int bits, int sym,
                           int n_grid, int n_cand, int32_t* tensor_q, uint16_t* scales_f16, int32_t* zeros);
/* awq.py:173-213 per group: scale / zero point as exact doubles [rows, G] */
int oracle_group_params(const void* x, int dtype, int64_t rows, int64_t K, int64_t L, int bits, int sym,
                        double* scales, double* zeros);
/* gpu = 1: as torch's GPU kernels evaluate awq.py:202-211 (reciprocal scale, +0 zero point) */
int oracle_group_params_ex(const void* x, int dtype, int64_t rows, int64_t K, int64_t L, int bits, int sym, int gpu,
                           double* scales, double* zeros);
/* awq.py:215-250 (mode 0) / 252-284 (mode 1) with given per-group parameters; out in dtype */
int oracle_apply_params(const void* x, int dtype, int64_t rows, int64_t K, int64_t L, const double* scales,
                        const double* zeros, int qmin, int qmax, int mode, void* out);
/* the same ops under torch's type promotion: x of dtype xdt (float or integer codes), first op
 * in d1, second in d2 (= out dtype; integer codes up to U8), one parameter per element; flags
 * bit 0 / 1: the scale / zero_point is a one-element operand (original value in a bf16 / fp16
 * op); bit 2 / 3: that parameter array holds int64 values (bit 4 / 5: uint64); bit 6: torch's
 * GPU clamp (clamp(-0, 0, qmax) = +0) */
enum { AWQ_ORACLE_I32 = 4, AWQ_ORACLE_I64 = 5, AWQ_ORACLE_I16 = 6, AWQ_ORACLE_I8 = 7, AWQ_ORACLE_U8 = 8,
       AWQ_ORACLE_BOOL = 9, AWQ_ORACLE_U16 = 10, AWQ_ORACLE_U32 = 11, AWQ_ORACLE_U64 = 12 };
int oracle_apply_params_ex(const void* x, int xdt, int64_t n, const double* scales, const double* zeros, int qmin,
                           int qmax, int mode, int d1, int d2, int flags, void* out);
int oracle_dequantize(const int32_t* tensor_q, const uint16_t* scales_f16, const int32_t* zeros,
                      int64_t rows, int64_t K, int64_t L, float* out);
int oracle_pack_rows(const int32_t* v, int64_t rows, int64_t n, int bits, int qmin, int32_t* packed);
int oracle_set_threads(int n);
/* activation-aware scale search (product definition, include/awq_hip.h awq_act_*) */
int oracle_act_stats(const void* x, int dtype, int64_t T, int64_t K, float* x_mean, float* x_sq);
int oracle_weight_colsum(const void* w, int dtype, int64_t R, int64_t K, int64_t L, double* partial);
int oracle_column_mean(const double* partial, int64_t nblk, int64_t K, double divisor, float* out);
int oracle_act_scale_table(const float* x_mean, const float* w_mean, int64_t K, int n_grid, float* table);
/* the table's power function (include/awq_hip.h awq_pow definition) */
double oracle_det_pow(double x, double r);
int oracle_act_search_losses(const void* w, int dtype, int64_t R, int64_t K, int64_t L, int bits, int sym,
                             const float* table, int n_grid, const float* x_sq, float* part, int64_t stride);
int oracle_act_search_select(const float* part, int n_grid, int64_t stride, double* losses, int32_t* best);
int oracle_apply_input_scale(const void* w, int dtype, int64_t R, int64_t K, const float* s, void* out);
uint16_t oracle_f32_to_bf16(float f);
float oracle_bf16_to_f32(uint16_t h);
uint16_t oracle_f32_to_f16(float f);
float oracle_f16_to_f32(uint16_t h);
#ifdef __cplusplus
}
#endif
#endif
